// kernels_xband.hip -- SpMV with x staged through LDS, one column band at a time.
//
// One workgroup (1024 threads, 16 waves) per block of <= 4096 rows, one
// workgroup per CU.  LDS: two x bands (2 x 16384 floats = 128 KiB) and the
// block's accumulators (4096 floats = 16 KiB).  Software pipeline, one barrier
// per band: while band p is applied from one buffer, slice p+1 (held in
// registers since two bands earlier, wide float4 loads) is written to the other
// while slice p+3 and the entries of band p+3 are in flight.  Each wave takes whole 64-entry
// chunks: term = x_lds[col] * (v * alpha), then the chunk's terms are added to
// the LDS accumulators in rank rounds (no two lanes touch one row in a round;
// no atomics).
// A row's terms are therefore added in ascending column order (bands ascend,
// ranks ascend inside a band), starting from beta*y: bit-identical to the
// reference.  Layout and its builder: xband.h / xband.cpp.
#include "sm_internal.h"
#include "xband.h"

#include <cstdlib>

namespace smamd {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Range-checked buffer descriptor (wave-uniform): loads past `bytes` read 0, so
// the prefetches below need no bounds branches (a branch around a load makes
// hipcc drain vmcnt before the next one and serialises the pipeline).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, uint64_t bytes) {
    const uint32_t n = bytes > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)bytes;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)n,
                                             0x00020000);
}
constexpr int kAuxNt = 2;   // non-temporal: entries are read once



// ABL (ablation, development only): bit 1 skips the apply, bit 2 the x slice loads,
// bit 4 the entry loads (values kept live so nothing upstream is dead-code removed).
// OPT (tuning variants): bit 1 pads the accumulator rows, bit 2 skips all-dummy chunks.
template <int THREADS, int BAND, int BROWS, int CAP, int MAXB, int ABL = 0, int OPT = 0>
__global__ __launch_bounds__(THREADS) void spmv_xband_kernel(
    int32_t n_rows, int32_t n_cols, int32_t block_rows, int32_t n_bands,
    const int32_t *__restrict__ chunk_start,
    const uint32_t *__restrict__ word, const float *__restrict__ val,
    const float *__restrict__ x, float *__restrict__ y, float alpha, float beta) {
    constexpr int kWaves = THREADS / 64;
    constexpr int kXv = BAND / (4 * THREADS);   // float4 per thread per band
    static_assert(kXv >= 1, "band too small for the workgroup");
    __shared__ __attribute__((aligned(16))) float xs[2][BAND];
    __shared__ float yacc[BROWS + BROWS / 32];   // OPT&1: one pad word per 32 rows
    auto yslot = [](uint32_t r) -> uint32_t { return (OPT & 1) ? r + (r >> 5) : r; };
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int32_t b = blockIdx.x;
    const int32_t r0 = b * block_rows;
    const int32_t nr = min(block_rows, n_rows - r0);
    const int32_t *csg = chunk_start + (int64_t)b * n_bands;
    const int32_t c_first = csg[0];
    const int32_t c_last = csg[n_bands];
    const __amdgpu_buffer_rsrc_t xr_src = rsrc(x, (uint64_t)n_cols * 4);
    const __amdgpu_buffer_rsrc_t w_src =
        rsrc(word + (int64_t)c_first * 64, (uint64_t)(c_last - c_first) * 256);
    const __amdgpu_buffer_rsrc_t v_src =
        rsrc(val + (int64_t)c_first * 64, (uint64_t)(c_last - c_first) * 256);
    // Chunk table window in registers: lane l holds cs[cw + l] and cs[cw + 64 + l]
    // (block-relative); scalar reads via readlane, reloaded every 64 bands.
    int32_t cw = 0;
    int32_t cs_lo = 0, cs_hi = 0;
    auto load_cs_window = [&](int32_t base) {
        cw = base;
        const int32_t i0 = min(base + lane, n_bands), i1 = min(base + 64 + lane, n_bands);
        cs_lo = csg[i0] - c_first;
        cs_hi = csg[i1] - c_first;
    };
    auto cs_at = [&](int32_t i) -> int32_t {   // i in [cw, cw + 128), wave-uniform
        const int32_t j = i - cw;
        return j < 64 ? __builtin_amdgcn_readlane(cs_lo, j) : __builtin_amdgcn_readlane(cs_hi, j - 64);
    };
    load_cs_window(0);

    auto load_slice = [&](int32_t p, float4 *xr) {
#pragma unroll
        for (int k = 0; k < kXv; ++k) {
            const uint32_t off = 4u * (uint32_t)(p * BAND + 4 * (tid + k * THREADS));
            u32x4 v = {off, off, off, off};
            if (!(ABL & 2)) v = __builtin_amdgcn_raw_buffer_load_b128(xr_src, off, 0, 0);
            xr[k] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y),
                                __uint_as_float(v.z), __uint_as_float(v.w));
        }
    };
    auto store_slice = [&](int buf, const float4 *xr) {
#pragma unroll
        for (int k = 0; k < kXv; ++k)
            *reinterpret_cast<float4 *>(&xs[buf][4 * (tid + k * THREADS)]) = xr[k];
    };
    // Chunk c of band p for this wave (c beyond the band -> dummy after the load).
    auto load_entries = [&](int32_t p, uint32_t *w, float *v) {
        const bool inb = p < n_bands;
        const int32_t c0 = inb ? cs_at(p) : 0;
        const int32_t c1 = inb ? cs_at(p + 1) : 0;
#pragma unroll
        for (int k = 0; k < CAP; ++k) {
            const int32_t c = c0 + wave + k * kWaves;
            const uint32_t off = 4u * (uint32_t)(c * 64 + lane);
            uint32_t wl = (uint32_t)(lane * 131) & 0x3fffu, vl = off;
            if (!(ABL & 4)) {
                wl = __builtin_amdgcn_raw_buffer_load_b32(w_src, off, 0, kAuxNt);
                vl = __builtin_amdgcn_raw_buffer_load_b32(v_src, off, 0, kAuxNt);
            }
            w[k] = c < c1 ? wl : kXbDummyWord;
            v[k] = __uint_as_float(vl);
        }
    };
    // All chunks of a band at once: every lane's x and round-0 accumulator reads
    // issue together (one LDS wait), rank-0 terms land, then the few lanes of
    // rank >= 1 re-read and add in rank order (program order within the wave;
    // chunks of one band never share a row across waves).
    auto apply_band = [&](const float *xb, const uint32_t *wa, const float *va) {
        float xv[CAP], yv[CAP];
        uint32_t rk[CAP], rl[CAP];
        bool live[CAP];
        bool more = false;
        int kmax = 0;   // chunks of this wave holding live entries (wave-uniform)
#pragma unroll
        for (int k = 0; k < CAP; ++k)
            if (!(OPT & 2) ||
                __any(((wa[k] >> kXbColBits) & ((1u << kXbRankBits) - 1u)) != kXbDummyRank))
                kmax = k + 1;
#pragma unroll
        for (int k = 0; k < CAP; ++k) {
            if (k >= kmax) { live[k] = false; rk[k] = 0; rl[k] = 0; xv[k] = 0.0f; yv[k] = 0.0f; continue; }
            rk[k] = (wa[k] >> kXbColBits) & ((1u << kXbRankBits) - 1u);
            live[k] = rk[k] != kXbDummyRank;
            const uint32_t cl = live[k] ? (wa[k] & ((1u << kXbColBits) - 1u)) : 0u;
            rl[k] = live[k] ? yslot(wa[k] >> (kXbColBits + kXbRankBits)) : 0u;
            xv[k] = xb[cl];
            yv[k] = yacc[rl[k]];
            more |= live[k] && rk[k] > 0;
        }
        float t[CAP];
#pragma unroll
        for (int k = 0; k < CAP; ++k) {
            if (k >= kmax) { t[k] = 0.0f; continue; }
            t[k] = __fmul_rn(xv[k], __fmul_rn(va[k], alpha));
            if (live[k] && rk[k] == 0) yacc[rl[k]] = __fadd_rn(yv[k], t[k]);
        }
        if (__any(more)) {
            for (uint32_t r = 1;; ++r) {
                bool again = false;
#pragma unroll
                for (int k = 0; k < CAP; ++k) {
                    if (live[k] && rk[k] == r) yacc[rl[k]] = __fadd_rn(yacc[rl[k]], t[k]);
                    again |= live[k] && rk[k] > r;
                }
                if (!__any(again)) break;
            }
        }
    };

    // Register rings with static roles (the band loop is unrolled by 4, so no
    // register ever moves -- a move would make hipcc wait for the load that
    // filled it): x slices in X0/X1 (slice q lives in X[q % 2]), entries in
    // E0..E3 (band q in E[q % 4]).
    float4 X0[kXv], X1[kXv];
    uint32_t W0[CAP], W1[CAP], W2[CAP], W3[CAP];
    float V0[CAP], V1[CAP], V2[CAP], V3[CAP];
    load_slice(0, X0);
    for (int32_t i = tid; i < nr; i += THREADS) {
        float v = y[r0 + i];
        if (beta != 1.0f) v = __fmul_rn(v, beta);
        yacc[yslot(i)] = v;
    }
    __syncthreads();   // cs[] visible
    load_entries(0, W0, V0);
    load_entries(1, W1, V1);
    load_entries(2, W2, V2);
    store_slice(0, X0);
    load_slice(1, X1);
    load_slice(2, X0);
    __syncthreads();

    // Band p: buffer p&1 holds slice p (visible); X[(p+1)%2] holds slice p+1.
    // One barrier per band: the stores of slice p+1 into buffer (p+1)&1 (freed
    // by the previous barrier) and this band's reads of buffer p&1 both finish
    // before it.  Slice p+3 reuses the register set just stored; entries of
    // band p+3 reuse the set of band p-1.  Loads past the last band read zeros
    // (range-checked descriptors) and are never applied.
    auto step = [&](int32_t p, float4 *xnext, uint32_t *wa, float *va, uint32_t *wl, float *vl) {
        if (p + 4 >= cw + 128) load_cs_window(p);   // every 124 bands (n_bands > 124 only)
        store_slice((p + 1) & 1, xnext);
        load_slice(p + 3, xnext);
        load_entries(p + 3, wl, vl);
        const float *xbuf = xs[p & 1];
        // Every chunk of the band is in registers: the builder guarantees at
        // most CAP chunks per wave per band (no loop of loads in the pipeline,
        // so hipcc can count vmcnt exactly).
        if (ABL & 1) {
#pragma unroll
            for (int k = 0; k < CAP; ++k) asm volatile("" ::"v"(wa[k]), "v"(va[k]));
        } else {
            apply_band(xbuf, wa, va);
        }
        __syncthreads();
    };
    for (int32_t p = 0; p < n_bands; p += 4) {
        step(p, X1, W0, V0, W3, V3);
        if (p + 1 >= n_bands) break;
        step(p + 1, X0, W1, V1, W0, V0);
        if (p + 2 >= n_bands) break;
        step(p + 2, X1, W2, V2, W1, V1);
        if (p + 3 >= n_bands) break;
        step(p + 3, X0, W3, V3, W2, V2);
    }
    for (int32_t i = tid; i < nr; i += THREADS) y[r0 + i] = yacc[yslot(i)];
}

}  // namespace

constexpr int kXbDefaultOpt = 0;

bool cap_fits(const XbandDev &xb, int cap) {
    return xb.max_chunks_per_band <= (int64_t)cap * (kXbThreads / 64);
}

hipError_t launch_spmv_xband(const XbandDev &xb, int32_t n_rows, int32_t n_cols, const float *x,
                             float *y, float alpha, float beta, hipStream_t s) {
    if (xb.n_blocks <= 0) return hipSuccess;
    if (xb.block_rows > kXbBlockRows || xb.band_cols != kXbBandCols ||
        xb.n_bands > kXbMaxBands)
        return hipErrorInvalidValue;
    const int waves = kXbThreads / 64;
    const int64_t cap = (xb.max_chunks_per_band + waves - 1) / waves;
    const char *abl_env = getenv("SM_XBAND_ABLATE");
    const int abl = abl_env ? atoi(abl_env) : 0;
    const char *opt_env = getenv("SM_XBAND_OPT");
    const int opt = opt_env ? atoi(opt_env) : kXbDefaultOpt;
    if (opt != kXbDefaultOpt && abl == 0 && cap_fits(xb, 2)) {   // development variants
        switch (opt) {
#define SM_XBO(O)                                                                                 \
    case O:                                                                                       \
        hipLaunchKernelGGL((spmv_xband_kernel<kXbThreads, kXbBandCols, kXbBlockRows, 2, kXbMaxBands, 0, O>), \
                           dim3((unsigned)xb.n_blocks), dim3(kXbThreads), 0, s, n_rows, n_cols,     \
                           xb.block_rows, xb.n_bands, xb.d_chunk_start, xb.d_word, xb.d_val, x, y, \
                           alpha, beta);                                                          \
        return hipGetLastError();
            SM_XBO(0) SM_XBO(1) SM_XBO(2) SM_XBO(3)
#undef SM_XBO
        default: return hipErrorInvalidValue;
        }
    }
    if (abl) {   // development-only ablations (never the product path)
        switch (abl) {
#define SM_XBA(A)                                                                                 \
    case A:                                                                                       \
        hipLaunchKernelGGL((spmv_xband_kernel<kXbThreads, kXbBandCols, kXbBlockRows, 2, kXbMaxBands, A>), \
                           dim3((unsigned)xb.n_blocks), dim3(kXbThreads), 0, s, n_rows, n_cols,     \
                           xb.block_rows, xb.n_bands, xb.d_chunk_start, xb.d_word, xb.d_val, x, y, \
                           alpha, beta);                                                          \
        break;
            SM_XBA(1) SM_XBA(2) SM_XBA(3) SM_XBA(4) SM_XBA(5) SM_XBA(6) SM_XBA(7)
#undef SM_XBA
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
#define SM_XB(C)                                                                               \
    hipLaunchKernelGGL((spmv_xband_kernel<kXbThreads, kXbBandCols, kXbBlockRows, C, kXbMaxBands>), \
                       dim3((unsigned)xb.n_blocks), dim3(kXbThreads), 0, s, n_rows, n_cols,     \
                       xb.block_rows, xb.n_bands, xb.d_chunk_start, xb.d_word, xb.d_val, x, y, alpha, beta)
    if (cap <= 1) SM_XB(1);
    else if (cap <= 2) SM_XB(2);
    else if (cap <= kXbMaxCap) SM_XB(4);
    else return hipErrorInvalidValue;
#undef SM_XB
    return hipGetLastError();
}

}  // namespace smamd
