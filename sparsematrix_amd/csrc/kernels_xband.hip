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

namespace smamd {
namespace {

template <int THREADS, int BAND, int BROWS, int CAP>
__global__ __launch_bounds__(THREADS) void spmv_xband_kernel(
    int32_t n_rows, int32_t n_cols, int32_t n_bands, const int32_t *__restrict__ chunk_start,
    const uint32_t *__restrict__ word, const float *__restrict__ val,
    const float *__restrict__ x, float *__restrict__ y, float alpha, float beta) {
    constexpr int kWaves = THREADS / 64;
    constexpr int kXv = BAND / (4 * THREADS);   // float4 per thread per band
    static_assert(kXv >= 1, "band too small for the workgroup");
    __shared__ __attribute__((aligned(16))) float xs[2][BAND];
    __shared__ float yacc[BROWS];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int32_t b = blockIdx.x;
    const int32_t r0 = b * BROWS;
    const int32_t nr = min(BROWS, n_rows - r0);
    const int32_t *cs = chunk_start + (int64_t)b * n_bands;

    auto load_slice = [&](int32_t p, float4 *xr) {
#pragma unroll
        for (int k = 0; k < kXv; ++k) {
            const int64_t c = (int64_t)p * BAND + 4 * (tid + k * THREADS);
            if (c + 3 < n_cols) {
                xr[k] = *reinterpret_cast<const float4 *>(x + c);
            } else {
                xr[k].x = c + 0 < n_cols ? x[c + 0] : 0.0f;
                xr[k].y = c + 1 < n_cols ? x[c + 1] : 0.0f;
                xr[k].z = c + 2 < n_cols ? x[c + 2] : 0.0f;
                xr[k].w = c + 3 < n_cols ? x[c + 3] : 0.0f;
            }
        }
    };
    auto store_slice = [&](int buf, const float4 *xr) {
#pragma unroll
        for (int k = 0; k < kXv; ++k)
            *reinterpret_cast<float4 *>(&xs[buf][4 * (tid + k * THREADS)]) = xr[k];
    };
    // Entries are read once: non-temporal loads keep them from evicting x in L2.
    auto load_entries = [&](int32_t p, uint32_t *w, float *v) {
        const int32_t c0 = p < n_bands ? cs[p] : 0;
        const int32_t c1 = p < n_bands ? cs[p + 1] : 0;
#pragma unroll
        for (int k = 0; k < CAP; ++k) {
            const int32_t c = c0 + wave + k * kWaves;
            if (c < c1) {
                w[k] = __builtin_nontemporal_load(word + (int64_t)c * 64 + lane);
                v[k] = __builtin_nontemporal_load(val + (int64_t)c * 64 + lane);
            } else {
                w[k] = kXbDummyWord;
                v[k] = 0.0f;
            }
        }
    };
    // One entry per lane of a chunk: term, then rank rounds into yacc.
    auto apply = [&](const float *xb, uint32_t w, float v) {
        const uint32_t rank = (w >> kXbColBits) & ((1u << kXbRankBits) - 1u);
        const bool live = rank != kXbDummyRank;
        const uint32_t cl = w & ((1u << kXbColBits) - 1u);
        const uint32_t rl = w >> (kXbColBits + kXbRankBits);
        const float t = __fmul_rn(xb[live ? cl : 0], __fmul_rn(v, alpha));
        for (uint32_t r = 0;; ++r) {
            if (live && rank == r) yacc[rl] = __fadd_rn(yacc[rl], t);
            if (!__any(live && rank > r)) break;
        }
    };

    // Prologue: accumulators = beta*y, slice 0 in buffer 0, slices 1 and 2 in
    // registers, entries of bands 0..2 in registers.
    float4 xa[kXv], xb2[kXv];
    uint32_t w0[CAP], w1[CAP], w2[CAP], w3[CAP];
    float v0[CAP], v1[CAP], v2[CAP], v3[CAP];
    load_slice(0, xa);
    load_entries(0, w0, v0);
    load_entries(1, w1, v1);
    load_entries(2, w2, v2);
    for (int32_t i = tid; i < nr; i += THREADS) {
        float v = y[r0 + i];
        if (beta != 1.0f) v = __fmul_rn(v, beta);
        yacc[i] = v;
    }
    store_slice(0, xa);
    if (n_bands > 1) load_slice(1, xa);
    if (n_bands > 2) load_slice(2, xb2);
    __syncthreads();

    // Band p: buffer p&1 holds slice p (visible); xa = slice p+1, xb2 = slice p+2.
    // One barrier per band: the stores of slice p+1 into buffer (p+1)&1 (freed
    // by the previous barrier) and this band's reads of buffer p&1 both finish
    // before it.  Loads run two bands (x) and three bands (entries) ahead.
    for (int32_t p = 0; p < n_bands; ++p) {
        if (p + 1 < n_bands) store_slice((p + 1) & 1, xa);
#pragma unroll
        for (int k = 0; k < kXv; ++k) xa[k] = xb2[k];
        if (p + 3 < n_bands) load_slice(p + 3, xb2);
        load_entries(p + 3, w3, v3);
        const float *xbuf = xs[p & 1];
#pragma unroll
        for (int k = 0; k < CAP; ++k) apply(xbuf, w0[k], v0[k]);
        // chunks beyond the prefetched CAP per wave (dense bands): load on demand
        for (int32_t c = cs[p] + wave + CAP * kWaves; c < cs[p + 1]; c += kWaves)
            apply(xbuf, word[(int64_t)c * 64 + lane], val[(int64_t)c * 64 + lane]);
#pragma unroll
        for (int k = 0; k < CAP; ++k) {
            w0[k] = w1[k]; v0[k] = v1[k];
            w1[k] = w2[k]; v1[k] = v2[k];
            w2[k] = w3[k]; v2[k] = v3[k];
        }
        __syncthreads();
    }
    for (int32_t i = tid; i < nr; i += THREADS) y[r0 + i] = yacc[i];
}

}  // namespace

hipError_t launch_spmv_xband(const XbandDev &xb, int32_t n_rows, int32_t n_cols, const float *x,
                             float *y, float alpha, float beta, hipStream_t s) {
    if (xb.n_blocks <= 0) return hipSuccess;
    if (xb.block_rows != kXbBlockRows || xb.band_cols != kXbBandCols) return hipErrorInvalidValue;
    hipLaunchKernelGGL((spmv_xband_kernel<kXbThreads, kXbBandCols, kXbBlockRows, 2>),
                       dim3((unsigned)xb.n_blocks), dim3(kXbThreads), 0, s, n_rows, n_cols,
                       xb.n_bands, xb.d_chunk_start, xb.d_word, xb.d_val, x, y, alpha, beta);
    return hipGetLastError();
}

}  // namespace smamd
