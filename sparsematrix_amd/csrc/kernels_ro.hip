// kernels_ro.hip -- SpMV over the row-owner codebook bands (ro.h, ro.cpp).
//
// One 1024-thread workgroup per tile (block of 16K rows x slab of columns), one per CU, as
// the balanced codebook bands (kernels_band2.hip): the block's row sums in LDS, x streamed
// through three 30 KiB LDS windows by LDS-DMA, the <= 255-entry table scaled by alpha in
// LDS (4 copies), the slab hand-off of xband_dev.h.  Roles:
//   waves 0..13 apply: wave w owns the block's rows [w * 1171, (w + 1) * 1171) and walks its
//     own chunk stream (ro.cpp) four chunks at a time, in window order, stage by stage (ro.h:
//     a stage's chunks have disjoint rows, so they are applied together);
//   waves 14..15 load: each issues half of every window's 30 1 KiB pieces.
// No barrier between windows: a wave applies window q's chunks once both loaders have
// published window q in LDS (ldp[] >= q + 1), and publishes prog[w] = q when it moves on to
// window q (it has read all of windows < q); a loader refills window q - 3's buffer once every
// applying wave's prog >= q - 2.  No two waves touch one row's sum, so the sums need no
// ordering between waves; inside a wave the chunks are applied in stream order, so each row's
// terms are added in ascending column order inside the slab (kernel.cc:780-796).
//
// Why (profiles/r05_dma3_phase_prof.txt, r05_xstream_*.txt): the barrier-synchronised bands of
// cband wait at every band for the slowest wave (~600 of ~1500 cycles per band), and one loader
// wave issues LDS-DMA at ~50 GB/s per CU, two at ~95.
#include "sm_internal.h"
#include "ro.h"
#include "xband.h"
#include "xband_dev.h"

#include <cstdio>
#include <cstdlib>

namespace smamd {
namespace {

constexpr int kRoThreads = 1024;
constexpr int kRoBufs = 3;
constexpr int kRoPieces = kRoWindow / 256;                       // 30
constexpr int kRoPpl = (kRoPieces + kRoLoadWaves - 1) / kRoLoadWaves;   // 15
constexpr int kRoTab = 4;                                         // table copies
constexpr uint32_t kRoColMask = (1u << 13) - 1u;
constexpr uint32_t kRoWinMask = (uint32_t)kRoMaxWindows - 1u;
constexpr int kRoOffShift = 13 + kCbIdBits;                       // 21
static_assert(kRoApplyWaves + kRoLoadWaves == kRoThreads / 64, "roles fill the workgroup");
static_assert(kRoPieces % kRoLoadWaves == 0, "whole pieces per loader");

#ifdef SM_DEV
// PROF (SM_RO_PROF=1, development): cycles per wave -- [0] prologue, [1] applying: waiting for
// the loaders, [2] applying: the rest of the chunk loop, [3] epilogue; [4] loader: waiting for
// the applying waves, [5] loader: DMA issue + landing; [6] pairs, [7] pairs applied in turn,
// [8] applying waves | loader waves << 32.
__device__ unsigned long long g_ro_prof[10];
#endif

constexpr int AE = 2;   // entry groups (kRoGroup chunks) in flight per applying wave

// ABL (development ablations, SM_RO_ABLATE, results wrong): 1 the loaders issue no DMA, 2 no x
// reads, 4 no sum reads or writes, 8 no apply at all, 16 no waits on the loaders.
template <bool PROF, int ABL>
__global__ __launch_bounds__(kRoThreads) void spmv_ro_kernel(
    int32_t n_rows, int32_t n_cols, int32_t n_slabs, int32_t slab_cols, const int32_t *__restrict__ wave_start,
    const uint32_t *__restrict__ ent, uint64_t ent_bytes, const float *__restrict__ table, int32_t table_size,
    const float *__restrict__ x, float *__restrict__ y, float *__restrict__ partials, int32_t *__restrict__ ctl,
    float alpha, float beta) {
    __shared__ __attribute__((aligned(16))) float xs[kRoBufs][kRoWindow];
    __shared__ __attribute__((aligned(16))) float yacc[kRoBlockRows];
    __shared__ float tab[256 * kRoTab];
    __shared__ int32_t prog[16];   // applying wave w: windows < prog[w] read in full
    __shared__ int32_t ldp[kRoLoadWaves];   // loader l: its pieces of windows < ldp[l] have landed
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    [[maybe_unused]] unsigned long long ph[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    [[maybe_unused]] unsigned long long tk = PROF ? clock64() : 0;
    auto mark = [&](int k) {
        if constexpr (PROF) {
            const unsigned long long now = clock64();
            ph[k] += now - tk;
            tk = now;
        }
    };
    const int32_t t = blockIdx.x;
    const int32_t b = t / n_slabs, slab = t - b * n_slabs;
    const uint64_t old_started = handoff_begin(ctl + (int64_t)b * kCtlWords, n_slabs);
    const int32_t r0 = b * kRoBlockRows;
    const int32_t nr = min(kRoBlockRows, n_rows - r0);
    const int32_t c0 = slab * slab_cols;
    const int32_t c1 = min(n_cols, c0 + slab_cols);
    const int32_t nq = (c1 - c0 + kRoWindow - 1) / kRoWindow;
    const __amdgpu_buffer_rsrc_t x_src = rsrc(x, (uint64_t)n_cols * 4);
    const uint32_t xs_lds = (uint32_t)(size_t)(__attribute__((address_space(3))) float *)&xs[0][0];
    auto lds_ld = [](const int32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    auto lds_st = [](int32_t *p, int32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };

    // Loader l's pieces (l, l + 2, ...) of window q into buffer q % 3; pieces past x read 0.
    const int ld = wid - kRoApplyWaves;
    auto dma_win = [&](int32_t q) {
        const int32_t cw = c0 + q * kRoWindow;
        const uint32_t buf = (uint32_t)(q % kRoBufs) * (uint32_t)kRoWindow;
#pragma unroll
        for (int k = 0; k < kRoPpl; ++k) {
            const int m = ld + k * kRoLoadWaves;
            const uint32_t voff = 4u * (uint32_t)(cw + m * 256 + lane * 4);
            const uint32_t lds = __builtin_amdgcn_readfirstlane(xs_lds + 4u * (buf + (uint32_t)m * 256u));
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(voff), "s"(x_src), "s"(lds)
                : "memory");
        }
    };

    // Prologue: the loaders' first windows go out first, then the applying waves' first entry
    // pairs, the table and (slab 0) y.
    const int32_t ws = wid < kRoApplyWaves ? wave_start[t * kRoApplyWaves + wid] : 0;
    const int32_t we = wid < kRoApplyWaves ? wave_start[t * kRoApplyWaves + wid + 1] : 0;
    const int32_t nch = we - ws;
    const __amdgpu_buffer_rsrc_t e_src = rsrc(ent, ent_bytes);
    // Entry of this lane in chunk i of the wave's stream (past the stream: 0 = a dummy).
    auto load_c = [&](int32_t i) -> uint32_t {
        const uint32_t off = i < nch ? 256u * (uint32_t)(ws + i) + 4u * (uint32_t)lane : 0xFFFFFFF0u;
        return __builtin_amdgcn_raw_buffer_load_b32(e_src, off, 0, kAuxNt);
    };
    if (wid >= kRoApplyWaves) {
        if constexpr (!(ABL & 1))
            for (int32_t q = 0; q < min(nq, 2); ++q) dma_win(q);
    }
    constexpr int G = kRoGroup;
    uint32_t E[AE][G];
    if (wid < kRoApplyWaves) {
#pragma unroll
        for (int v = 0; v < AE; ++v)
#pragma unroll
            for (int k = 0; k < G; ++k) E[v][k] = load_c(G * v + k);
    }
    {   // table: fl(table[id] * alpha), four copies, id 255 (dummies) and past the table 0
        const int id = tid >> 2;
        tab[tid] = id < table_size ? __fmul_rn(table[id], alpha) : 0.0f;
    }
    constexpr int kQ = kRoBlockRows / (4 * kRoThreads);
    const bool y_vec = ((uintptr_t)(y + r0) & 15) == 0;
    if (slab == 0) {
        const __amdgpu_buffer_rsrc_t yi_src = rsrc(y + r0, (uint64_t)nr * 4);
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const uint32_t o = 16u * (uint32_t)(tid + q * kRoThreads);
            float4 v;
            if (y_vec) {
                const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(yi_src, o, 0, 0);
                v = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
            } else {
                v = make_float4(__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o, 0, 0)),
                                __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 4, 0, 0)),
                                __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 8, 0, 0)),
                                __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 12, 0, 0)));
            }
            if (beta != 1.0f) v = make_float4(__fmul_rn(v.x, beta), __fmul_rn(v.y, beta), __fmul_rn(v.z, beta), __fmul_rn(v.w, beta));
            *reinterpret_cast<float4 *>(&yacc[4 * (tid + q * kRoThreads)]) = v;
        }
    } else {
#pragma unroll
        for (int q = 0; q < kQ; ++q)
            *reinterpret_cast<float4 *>(&yacc[4 * (tid + q * kRoThreads)]) = make_float4(-0.f, -0.f, -0.f, -0.f);
    }
    if (tid < 16) prog[tid] = 0;
    if (tid < kRoLoadWaves) ldp[tid] = 0;
    __syncthreads();
    const uint64_t snap = handoff_snapshot(ctl + (int64_t)b * kCtlWords, n_slabs);
    mark(0);

    if (wid >= kRoApplyWaves) {
        // ---- loader ------------------------------------------------------------------
        // Issue the next window as soon as its buffer is free (every applying wave has moved
        // past the window it held), else publish the oldest window in flight once it lands:
        // a wave reading window p may so have p + 1 and p + 2 landed beside it.
        __builtin_amdgcn_s_setprio(3);
        int32_t issued = min(nq, 2), landed = 0;
        while (landed < nq) {
            bool can = false;
            if (issued < nq) {
                if (issued < kRoBufs) {
                    can = true;
                } else {   // buffer issued % 3 held window issued - 3
                    const int32_t need = issued - 2;
                    mark(5);
                    const int32_t p = lane < kRoApplyWaves ? lds_ld(&prog[lane]) : need;
                    can = __ballot(p < need) == 0;
                    mark(4);
                }
            }
            if (can) {
                if constexpr (!(ABL & 1)) dma_win(issued);
                ++issued;
                continue;
            }
            const int32_t out = issued - landed;   // windows in flight, oldest first
            if (out == 0) {
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            if (out >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kRoPpl) : "memory");
            else if (out == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kRoPpl) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ++landed;
            if (lane == 0) lds_st(&ldp[ld], landed);
        }
        mark(5);
        ph[8] = 1ull << 32;
    } else {
        // ---- applying wave -----------------------------------------------------------
        const int32_t wrow = wid * kRoWaveRows;   // the wave's first row in the block
        const uint32_t dmy = kCbDummyWord;
        int32_t done_q = 0;   // published: windows < done_q read in full
        int32_t ready = 0;    // windows < ready landed (both loaders)
        auto shr1 = [](float v) {   // lane i <- lane i-1 (lane 0 <- 0)
            return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, false));
        };
        auto sel = [](uint64_t m, float a, float bb) -> float {
            float r;
            asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(bb), "s"(m));
            return r;
        };
        const int32_t ngrp = (nch + G - 1) / G;
        const int32_t ngu = (ngrp + AE - 1) / AE * AE;
        for (int32_t g0 = 0; g0 < ngu; g0 += AE) {
#pragma unroll
            for (int u = 0; u < AE; ++u) {
                const int32_t gi = g0 + u;
                if (gi < ngrp) {   // wave-uniform
                    uint32_t wd[G], qk[G], st[G], base[G];
                    uint32_t qmax = 0, smax = 0;
#pragma unroll
                    for (int k = 0; k < G; ++k) {
                        wd[k] = E[u][k] ^ dmy;
                        const uint32_t h = (uint32_t)__builtin_amdgcn_readlane((int)wd[k], 0);
                        qk[k] = h & kRoWinMask;
                        st[k] = (h >> kRoStageShift) & 3u;
                        base[k] = (uint32_t)wrow + (((h >> kRoOffShift) & kCbOffMask) | ((h >> kCbContBit) << 10));
                        if (k > 0 && G * gi + k >= nch) { qk[k] = qk[0]; st[k] = 0; }   // past the stream: a dummy
                        qmax = max(qmax, qk[k]);
                        smax = max(smax, st[k]);
                    }
                    // Stage by stage (each stage's chunks have disjoint rows), all windows of the
                    // group landed first -- unless the group spans more windows than the ring
                    // holds ahead of its first (the loaders refill window q only once every wave
                    // has moved to q - 2): then chunk by chunk, publishing as it goes.
                    const bool serial = qmax > qk[0] + 2;
                    const int npass = serial ? G : (int)smax + 1;
                    if constexpr (PROF) {
                        ph[6] += 1;
                        ph[7] += (unsigned long long)(npass - 1);
                    }
                    for (int ps = 0; ps < npass; ++ps) {
                        uint32_t qps = qk[0];   // qk[ps], without a dynamically indexed array
#pragma unroll
                        for (int k = 1; k < G; ++k) qps = k == ps ? qk[k] : qps;
                        const uint32_t qlo = serial ? qps : qk[0], qhi = serial ? qps : qmax;
                        if ((int32_t)qlo > done_q) {   // moving on: windows < qlo are read in full
                            done_q = (int32_t)qlo;
                            if (lane == 0) lds_st(&prog[wid], done_q);
                        }
                        mark(2);
                        while (!(ABL & 16) && ready <= (int32_t)qhi) {   // both loaders' pieces of window qhi
                            const int32_t a = lds_ld(&ldp[0]), bb = lds_ld(&ldp[1]);
                            ready = min(a, bb);
                            if (ready <= (int32_t)qhi) __builtin_amdgcn_s_sleep(1);
                        }
                        mark(1);
                        if constexpr (ABL & 8) continue;
                        __builtin_amdgcn_s_setprio(2);
                        float xv[G], tv[G], yv[G];
                        uint32_t rl[G];
                        uint64_t live[G], cont[G];
#pragma unroll
                        for (int k = 0; k < G; ++k) {
                            const uint64_t on = (serial ? k == ps : st[k] == (uint32_t)ps) ? ~1ull : 0ull;
                            const uint32_t id = (wd[k] >> 13) & kCbDummyId;
                            live[k] = __ballot(id != kCbDummyId) & on;
                            cont[k] = __ballot((int32_t)wd[k] < 0) & on;
                            rl[k] = base[k] + ((wd[k] >> kRoOffShift) & kCbOffMask);
                            xv[k] = (ABL & 2) ? 1.0f : xs[qk[k] % kRoBufs][wd[k] & kRoColMask];
                            tv[k] = tab[id * kRoTab + (lane & (kRoTab - 1))];
                            yv[k] = (ABL & 4) ? 0.0f : yacc[min(rl[k], (uint32_t)(kRoBlockRows - 1))];
                        }
                        asm volatile("" : "+v"(xv[0]), "+v"(xv[1]), "+v"(xv[2]), "+v"(xv[3]), "+v"(yv[0]), "+v"(yv[1]),
                                     "+v"(yv[2]), "+v"(yv[3]), "+v"(tv[0]), "+v"(tv[1]), "+v"(tv[2]), "+v"(tv[3]));
                        float tm[G], acc[G];
                        uint64_t R[G];
#pragma unroll
                        for (int k = 0; k < G; ++k) {
                            tm[k] = __fmul_rn(xv[k], tv[k]);
                            acc[k] = __fadd_rn(yv[k], tm[k]);
                            R[k] = cont[k] & ~(cont[k] << 1);
                        }
                        while ((R[0] | R[1] | R[2] | R[3]) != 0) {
#pragma unroll
                            for (int k = 0; k < G; ++k) {
                                acc[k] = sel(R[k], acc[k], __fadd_rn(shr1(acc[k]), tm[k]));
                                R[k] = cont[k] & (R[k] << 1);
                            }
                        }
#pragma unroll
                        for (int k = 0; k < G; ++k) {   // the segment's last lane writes its row
                            const uint64_t last = live[k] & ~(cont[k] >> 1);
                            if (!(ABL & 4) && ((last >> lane) & 1)) yacc[rl[k]] = acc[k];
                        }
                        __builtin_amdgcn_s_setprio(0);
                    }
                }
#pragma unroll
                for (int k = 0; k < G; ++k) E[u][k] = load_c(G * (gi + AE) + k);
            }
        }
        if (lane == 0) lds_st(&prog[wid], nq);   // every window read
        mark(2);
        ph[8] = 1;
    }
    auto flush = [&]() {
#ifdef SM_DEV
        if constexpr (PROF) {
            mark(3);
            if (lane == 0) {
                for (int k = 0; k < 8; ++k) atomicAdd(&g_ro_prof[k], ph[k]);
                atomicAdd(&g_ro_prof[8], ph[8]);
            }
        }
#endif
    };
    __syncthreads();   // every wave done: the sums are final, the hand-off words live in xs
    if (n_slabs == 1) {
        const int32_t nv = y_vec ? (nr & ~3) : 0;
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int32_t i = 4 * (tid + q * kRoThreads);
            if (i < nv) *reinterpret_cast<float4 *>(y + r0 + i) = *reinterpret_cast<const float4 *>(&yacc[i]);
        }
        for (int32_t i = nv + tid; i < nr; i += kRoThreads) y[r0 + i] = yacc[i];
        flush();
        return;
    }
    int32_t *s_word = reinterpret_cast<int32_t *>(&xs[0][0]);
    slab_handoff_epoch<kRoThreads>(yacc, ctl + (int64_t)b * kCtlWords, s_word, y, partials, n_rows, r0, nr, slab,
                                   n_slabs, y_vec, old_started, snap);
    flush();
}

}  // namespace

// XbandDev of kind kXbRo: d_chunk_start = the (tile, wave) chunk starts, d_word = the chunks,
// slab_bands = columns per slab, n_chunks = chunks.
hipError_t launch_spmv_ro(const XbandDev &d, int32_t n_rows, int32_t n_cols, const float *x, float *y,
                          float alpha, float beta, hipStream_t s) {
    if (d.n_blocks <= 0) return hipSuccess;
    if (d.kind != kXbRo || !d.d_chunk_start || !d.d_word || !d.d_table || d.table_size < 0 ||
        d.table_size > (int32_t)kCbDummyId || d.block_rows > kRoBlockRows || (d.n_slabs > 1 && (!d.d_partials || !d.d_tickets)))
        return hipErrorInvalidValue;
#define SM_RO(P, A)                                                                                 \
    hipLaunchKernelGGL((spmv_ro_kernel<P, A>), dim3((unsigned)((int64_t)d.n_blocks * d.n_slabs)), dim3(kRoThreads), 0, s, \
                       n_rows, n_cols, d.n_slabs, d.slab_bands, d.d_chunk_start, d.d_word,             \
                       (uint64_t)d.n_chunks * 256u, d.d_table, d.table_size, x, y, d.d_partials, d.d_tickets, \
                       alpha, beta)
#ifdef SM_DEV
    static const bool prof = [] {
        const char *e = dev_env("SM_RO_PROF");
        return e && atoi(e) != 0;
    }();
    static const int abl = [] {
        const char *e = dev_env("SM_RO_ABLATE");
        return e ? atoi(e) : 0;
    }();
#define SM_RO_ABL(P)                                                                                \
    switch (abl) {                                                                                  \
    case 0: SM_RO(P, 0); break;                                                                     \
    case 1: SM_RO(P, 1); break;                                                                     \
    case 2: SM_RO(P, 2); break;                                                                     \
    case 4: SM_RO(P, 4); break;                                                                     \
    case 6: SM_RO(P, 6); break;                                                                     \
    case 8: SM_RO(P, 8); break;                                                                     \
    case 16: SM_RO(P, 16); break;                                                                   \
    case 25: SM_RO(P, 25); break;                                                                   \
    default: return hipErrorInvalidValue;                                                           \
    }
    if (prof) {
        unsigned long long h[10] = {};
        void *sym = nullptr;
        if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_ro_prof)) != hipSuccess) return hipErrorInvalidValue;
        (void)hipMemsetAsync(sym, 0, sizeof(h), s);
        SM_RO_ABL(true)
        (void)hipMemcpyAsync(h, sym, sizeof(h), hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        const double wa = (double)(h[8] & 0xFFFFFFFFull), wl = (double)(h[8] >> 32);
        fprintf(stderr, "ro prof abl %d (cycles per wave; %.0f applying + %.0f loader waves; %.1f pairs, %.1f in turn per "
                "applying wave): applying: prologue %.0f loader wait %.0f chunks %.0f epilogue %.0f | loaders: "
                "wait %.0f dma %.0f\n", abl, wa, wl, h[6] / wa, h[7] / wa, h[0] / (wa + wl), h[1] / wa, h[2] / wa,
                h[3] / (wa + wl), h[4] / wl, h[5] / wl);
        return hipGetLastError();
    }
    if (abl != 0) {
        SM_RO_ABL(false)
        return hipGetLastError();
    }
#undef SM_RO_ABL
#endif
    SM_RO(false, 0);
#undef SM_RO
    return hipGetLastError();
}

}  // namespace smamd
