// kernels_gcb.hip -- SpMV over the gathered chunk bands (gcb.h, gcb.cpp): wide matrices
// whose x cannot be staged (BASELINE config 5's rank slices, x = 256 MiB).
//
// One 1024-thread workgroup (16 waves) per tile = (block of 2^ROWS_LOG2 rows, slab of
// columns); the block's sums live in LDS (128 KiB at 32K rows).  Per band p, every wave:
//   gathers the x values of band p+GA (its words arrived ER-GA bands ago) straight from
//     memory -- one 4-byte load per term, dummy and header lanes send no request;
//   applies band p: decodes its two chunks (lane 0's header = the chunk's base row),
//     reads the rows' sums, adds x * fl(v * alpha) with the running sum of a row's
//     segment passed up consecutive lanes by DPP (rank rounds on SGPR lane masks, as the
//     cband kernel), and the segment's last lane writes the row;
//   loads the 16-byte entry slot of band p+ER into the registers band p just freed;
//   barrier (a row's next terms may sit in another wave's chunk of the next band).
// A band holds up to 2016 terms, so the per-band barrier and latency chain are paid
// ~8x less often per term than the gather-band kind's 32K-column bands of 128 terms on
// config 5's slice (kernels_xband.hip spmv_gband_kernel: 2 of its 16 waves had work).
//
// Summation order: within a tile every row's terms ascend in column (gcb.h); slab 0 starts
// from beta*y, later slabs from -0.0, and the slab sums are added in slab order by the
// blocked kinds' hand-off (xband_dev.h) -- bit-identical to the reference with one slab
// (kernel.cc:780-796, :791), within the Sum|terms| bound otherwise, deterministic always.
#include "gcb.h"
#include "sm_internal.h"
#include "xband.h"
#include "xband_dev.h"

namespace smamd {
namespace {

constexpr int kGcbThreads = 1024;

// ABL (development builds, SM_GCB_ABLATE; results wrong): 1 no x gathers (x read as 0,
// no memory request), 2 no apply (the loaded values kept live), 4 no per-band barrier.
// PACE: column pacing (below), a development A/B until measured.
// XAUX: cache-policy bits of the x gathers (development A/B).
template <int ROWS_LOG2, int ER, int GA, int ABL = 0, bool PACE = false, int XAUX = 0>
__global__ __launch_bounds__(kGcbThreads) void spmv_gcb_kernel(
    int32_t n_rows, int32_t n_cols, int32_t block_rows, int32_t n_slabs,
    const int32_t *__restrict__ tile_band_start, const int32_t *__restrict__ band_clo,
    const uint32_t *__restrict__ ent, const float *__restrict__ x, float *__restrict__ y,
    float *__restrict__ partials, int32_t *__restrict__ ctl, float alpha, float beta,
    int32_t *__restrict__ pace, int32_t pace_k, int32_t pace_slack) {
    constexpr int BROWS = 1 << ROWS_LOG2;
    constexpr int XR = GA + 1;                  // x-value ring: band p's slot is not refilled at p
    constexpr int U = ER % XR == 0 ? ER : ER * XR;   // unroll: static ring roles
    static_assert(GA >= 1 && GA < ER, "gathers need the entries of their band");
    static_assert(BROWS % (4 * kGcbThreads) == 0, "accumulator init in float4 per thread");
    __shared__ __attribute__((aligned(16))) float yacc[BROWS];
    __shared__ int32_t s_word[4];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int32_t t = blockIdx.x;
    const int32_t b = t / n_slabs;
    const int32_t slab = t - b * n_slabs;
    handoff_started(ctl + (int64_t)b * kCtlWords, n_slabs);
    // Column pacing (pace != null): the tiles of one dispatch group (blockIdx mod 8: one XCD
    // under round-robin dealing, for speed only) sweep the columns together, so the x lines
    // one tile gathers are still in the XCD's L2 when the group's other tiles reach them.  A
    // tile adds 1 to checkpoint k's counter when its bands pass column k * 2^18, and before
    // going past checkpoint k waits until every STARTED tile of its group has passed
    // k - slack -- the slowest tile never waits, so the group always progresses.  Counters
    // are monotonic across launches (launches on a matrix are ordered): this launch's counts
    // are the values minus gen_base = launch index * group size.
    const int32_t pg = (int32_t)(blockIdx.x & 7u);
    const int32_t pn = ((int32_t)gridDim.x - pg + 7) / 8;   // tiles in the group
    int32_t *pw = PACE ? pace + (int64_t)pg * (1 + pace_k) : nullptr;
    int32_t gen_base = 0, kdone = -1;
    if (PACE && tid == 0)
        gen_base = __hip_atomic_fetch_add(pw, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) / pn * pn;
    const int32_t g0 = tile_band_start[t];
    const int32_t nb = tile_band_start[t + 1] - g0;
    const int32_t r0 = b * block_rows;
    const int32_t nr = min(block_rows, n_rows - r0);
    const __amdgpu_buffer_rsrc_t x_src = rsrc(x, (uint64_t)n_cols * 4);
    const __amdgpu_buffer_rsrc_t e_src =
        rsrc(ent + (int64_t)g0 * kGcbBandWords, (uint64_t)nb * kGcbBandWords * 4);
    // Band windows: lane l holds clo of bands cw + l (lo) and cw + 64 + l (hi); the
    // window moves on when the band gathered next leaves its low half.
    const int32_t *clg = band_clo + g0;
    int32_t cw = 0;
    int32_t clo_lo = lane < nb ? clg[lane] : 0;
    int32_t clo_hi = 64 + lane < nb ? clg[64 + lane] : 0;
    auto clo_at = [&](int32_t q) -> int32_t {   // q in [cw, cw + 128), wave-uniform
        const int32_t j = q - cw;
        const int32_t lo = __builtin_amdgcn_readlane(clo_lo, j & 63);
        const int32_t hi = __builtin_amdgcn_readlane(clo_hi, j & 63);
        return j < 64 ? lo : hi;
    };
    auto advance = [&]() {
        cw += 64;
        clo_lo = clo_hi;
        clo_hi = cw + 64 + lane < nb ? clg[cw + 64 + lane] : 0;
    };
    // Entries of band q for this lane: {word 2w, word 2w+1, value 2w, value 2w+1};
    // past the tile: zeros = dummies (no memory request).
    auto load_e = [&](int32_t q) -> u32x4 {
        const uint32_t off = q < nb ? (uint32_t)kGcbBandWords * 4u * (uint32_t)q + 16u * (uint32_t)tid
                                    : 0xFFFFFFF0u;
        return __builtin_amdgcn_raw_buffer_load_b128(e_src, off, 0, kAuxNt);
    };
    // x of band q's two terms; dummies and headers read nothing (offset past the range).
    auto gather = [&](int32_t q, u32x4 e, float *xv) {
        const int32_t c = q < nb ? clo_at(q) : 0;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t w = e[k];
            const uint32_t off = ((w & kGcbLive) && !(ABL & 1)) ? 4u * (uint32_t)(c + (int32_t)(w & kGcbColMask))
                                                                : 0xFFFFFFF0u;
            xv[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(x_src, off, 0, XAUX));
        }
    };
    auto shr1 = [](float v) {   // lane i <- lane i-1
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, false));
    };
    auto sel = [](uint64_t m, float a, float bb) -> float {   // lane i: bb where bit i of m, else a
        float r;
        asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(bb), "s"(m));
        return r;
    };
    auto apply = [&](u32x4 e, const float *xv) {
        __builtin_amdgcn_s_setprio(2);
        float yv[2], tm[2], acc[2];
        uint32_t rl[2];
        uint64_t live[2], cont[2], R[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t w = e[k];
            const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)w, 0) & kGcbColMask;
            live[k] = __ballot((w & kGcbLive) != 0);
            cont[k] = __ballot((w & kGcbCont) != 0);
            rl[k] = base + ((w >> kGcbColBits) & kGcbOffMask);   // dummies: the base row (read only)
            yv[k] = yacc[rl[k]];
        }
        asm volatile("" : "+v"(yv[0]), "+v"(yv[1]));   // both reads before any write
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            tm[k] = __fmul_rn(xv[k], __fmul_rn(__uint_as_float(e[2 + k]), alpha));
            acc[k] = __fadd_rn(yv[k], tm[k]);
            R[k] = cont[k] & ~(cont[k] << 1);
        }
        while ((R[0] | R[1]) != 0) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                acc[k] = sel(R[k], acc[k], __fadd_rn(shr1(acc[k]), tm[k]));
                R[k] = cont[k] & (R[k] << 1);
            }
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {   // the segment's last lane writes its row
            const uint64_t last = live[k] & ~(cont[k] >> 1);
            if ((last >> lane) & 1) yacc[rl[k]] = acc[k];
        }
        __builtin_amdgcn_s_setprio(0);
    };

    // Prologue (virtual bands -U..-1 in the loop's order): entries of bands 0..ER-1, x of
    // bands 0..GA-1, then the accumulators (beta * y on slab 0, -0.0 on the others).
    u32x4 E[ER];
    float XV[XR][2];
#pragma unroll
    for (int v = 0; v < ER; ++v) E[v] = load_e(v);
#pragma unroll
    for (int v = 0; v < GA; ++v) gather(v, E[v], XV[v]);
    constexpr int kQ = BROWS / (4 * kGcbThreads);
    const bool y_vec = ((uintptr_t)(y + r0) & 15) == 0;
    if (slab == 0) {
        const __amdgpu_buffer_rsrc_t yi_src = rsrc(y + r0, (uint64_t)nr * 4);
        float4 yv[kQ];
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const uint32_t o = 16u * (uint32_t)(tid + q * kGcbThreads);
            if (y_vec) {
                const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(yi_src, o, 0, 0);
                yv[q] = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z),
                                    __uint_as_float(u.w));
            } else {
                yv[q] = make_float4(__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o, 0, 0)),
                                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 4, 0, 0)),
                                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 8, 0, 0)),
                                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 12, 0, 0)));
            }
        }
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            if (beta != 1.0f)
                yv[q] = make_float4(__fmul_rn(yv[q].x, beta), __fmul_rn(yv[q].y, beta),
                                    __fmul_rn(yv[q].z, beta), __fmul_rn(yv[q].w, beta));
            *reinterpret_cast<float4 *>(&yacc[4 * (tid + q * kGcbThreads)]) = yv[q];
        }
    } else {
#pragma unroll
        for (int q = 0; q < kQ; ++q)
            *reinterpret_cast<float4 *>(&yacc[4 * (tid + q * kGcbThreads)]) = make_float4(-0.f, -0.f, -0.f, -0.f);
    }
    __syncthreads();

    // Whole groups of U bands (static ring roles); steps past the tile see dummies only
    // and skip the barrier (a uniform branch).
    const int32_t nbu = (nb + U - 1) / U * U;
    for (int32_t p = 0; p < nbu; p += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t q = p + u;
            if (q + GA >= cw + 64) advance();   // the gather below reads clo of band q + GA
            if (PACE && tid == 0 && q + GA < nb) {   // checkpoints passed by the band gathered next
                const int32_t kq = min(clo_at(q + GA) >> kGcbColBits, pace_k - 1);
                for (int32_t k = kdone + 1; k <= kq; ++k)
                    __hip_atomic_fetch_add(pw + 1 + k, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (kq > kdone && kq >= pace_slack) {
                    const int32_t kw = kq - pace_slack;
                    for (;;) {
                        const int32_t st = min(pn, __hip_atomic_load(pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - gen_base);
                        const int32_t ar = __hip_atomic_load(pw + 1 + kw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - gen_base;
                        if (ar >= st) break;
                        __builtin_amdgcn_s_sleep(8);
                    }
                }
                kdone = max(kdone, kq);
            }
            gather(q + GA, E[(u + GA) % ER], XV[(u + GA) % XR]);
            if constexpr (ABL & 2) {
                asm volatile("" ::"v"(E[u % ER].x), "v"(E[u % ER].y), "v"(E[u % ER].z), "v"(E[u % ER].w),
                             "v"(XV[u % XR][0]), "v"(XV[u % XR][1]));
            } else {
                apply(E[u % ER], XV[u % XR]);
            }
            E[u % ER] = load_e(q + ER);
            if (!(ABL & 4) && q < nb) __syncthreads();
        }
    }

    if (PACE && tid < 64) {   // every checkpoint not yet passed, so the counts stay per launch
        const int32_t kd = __builtin_amdgcn_readfirstlane(kdone);
        for (int32_t k = kd + 1 + tid; k < pace_k; k += 64)
            __hip_atomic_fetch_add(pw + 1 + k, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (n_slabs == 1) {
        const int32_t nv = y_vec ? (nr & ~3) : 0;   // float4 rows, then the rest
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int32_t i = 4 * (tid + q * kGcbThreads);
            if (i < nv) *reinterpret_cast<float4 *>(y + r0 + i) = *reinterpret_cast<const float4 *>(&yacc[i]);
        }
        for (int32_t i = nv + tid; i < nr; i += kGcbThreads) y[r0 + i] = yacc[i];
        return;
    }
    slab_handoff<kGcbThreads>(yacc, ctl + (int64_t)b * kCtlWords, s_word, y, partials, n_rows, r0, nr,
                              slab, n_slabs, y_vec);
}

}  // namespace

hipError_t launch_spmv_gcb(const XbandDev &xb, int32_t n_rows, int32_t n_cols, const float *x, float *y,
                           float alpha, float beta, hipStream_t s) {
    if (xb.n_blocks <= 0) return hipSuccess;
    if (xb.kind != kXbGcb || xb.n_slabs < 1 || !xb.d_chunk_start || !xb.d_band_clo ||
        (xb.n_bands > 0 && !xb.d_word) || (xb.n_slabs > 1 && (!xb.d_partials || !xb.d_tickets)) ||
        xb.block_rows > (1 << 15))
        return hipErrorInvalidValue;
    const dim3 grid((unsigned)((int64_t)xb.n_blocks * xb.n_slabs)), block(kGcbThreads);
#define SM_GCB(RL, ER, GA)                                                                         \
    hipLaunchKernelGGL((spmv_gcb_kernel<RL, ER, GA>), grid, block, 0, s, n_rows, n_cols, xb.block_rows, \
                       xb.n_slabs, xb.d_chunk_start, xb.d_band_clo, xb.d_word, x, y, xb.d_partials,  \
                       xb.d_tickets, alpha, beta, pace, xb.pace_k, pace_slack)
    int look = 0;
    int32_t *pace = nullptr;
    int32_t pace_slack = 0;
    const bool tall = xb.block_rows > (1 << 14);
#ifdef SM_DEV
    if (const char *e = dev_env("SM_GCB_LOOK")) look = atoi(e);   // development A/B of ER/GA
    if (const char *e = dev_env("SM_GCB_XAUX")) {   // x gather cache policy (A/B)
        const int a = atoi(e);
#define SM_GCBX(A)                                                                                 \
    if (tall) hipLaunchKernelGGL((spmv_gcb_kernel<15, 6, 2, 0, false, A>), grid, block, 0, s, n_rows, n_cols,    \
                                 xb.block_rows, xb.n_slabs, xb.d_chunk_start, xb.d_band_clo, xb.d_word, x, y,  \
                                 xb.d_partials, xb.d_tickets, alpha, beta, nullptr, 0, 0);                   \
    else hipLaunchKernelGGL((spmv_gcb_kernel<14, 6, 2, 0, false, A>), grid, block, 0, s, n_rows, n_cols,         \
                            xb.block_rows, xb.n_slabs, xb.d_chunk_start, xb.d_band_clo, xb.d_word, x, y,       \
                            xb.d_partials, xb.d_tickets, alpha, beta, nullptr, 0, 0)
        switch (a) {
        case 1: SM_GCBX(1); break;
        case 2: SM_GCBX(2); break;
        case 16: SM_GCBX(16); break;
        case 17: SM_GCBX(17); break;
        default: SM_GCBX(0); break;
        }
#undef SM_GCBX
        return hipGetLastError();
    }
    if (const char *e = dev_env("SM_GCB_PACE")) {   // column pacing, slack in checkpoints (A/B)
        pace_slack = atoi(e);
        if (pace_slack > 0 && xb.d_pace) pace = xb.d_pace;
    }
    if (const char *e = dev_env("SM_GCB_ABLATE")) {
        const int abl = atoi(e);
#define SM_GCBA(A)                                                                                    \
    if (tall) hipLaunchKernelGGL((spmv_gcb_kernel<15, 6, 2, A>), grid, block, 0, s, n_rows, n_cols, xb.block_rows, \
                                 xb.n_slabs, xb.d_chunk_start, xb.d_band_clo, xb.d_word, x, y, xb.d_partials,  \
                                 xb.d_tickets, alpha, beta, pace, xb.pace_k, pace_slack);            \
    else hipLaunchKernelGGL((spmv_gcb_kernel<14, 6, 2, A>), grid, block, 0, s, n_rows, n_cols, xb.block_rows, \
                            xb.n_slabs, xb.d_chunk_start, xb.d_band_clo, xb.d_word, x, y, xb.d_partials,  \
                            xb.d_tickets, alpha, beta, pace, xb.pace_k, pace_slack)
        switch (abl) {
        case 1: SM_GCBA(1); break;
        case 2: SM_GCBA(2); break;
        case 3: SM_GCBA(3); break;
        case 4: SM_GCBA(4); break;
        case 5: SM_GCBA(5); break;
        default: return hipErrorInvalidValue;
        }
#undef SM_GCBA
        return hipGetLastError();
    }
#endif
    if (pace) {
        if (tall)
            hipLaunchKernelGGL((spmv_gcb_kernel<15, 6, 2, 0, true>), grid, block, 0, s, n_rows, n_cols, xb.block_rows,
                               xb.n_slabs, xb.d_chunk_start, xb.d_band_clo, xb.d_word, x, y, xb.d_partials,
                               xb.d_tickets, alpha, beta, pace, xb.pace_k, pace_slack);
        else
            hipLaunchKernelGGL((spmv_gcb_kernel<14, 6, 2, 0, true>), grid, block, 0, s, n_rows, n_cols, xb.block_rows,
                               xb.n_slabs, xb.d_chunk_start, xb.d_band_clo, xb.d_word, x, y, xb.d_partials,
                               xb.d_tickets, alpha, beta, pace, xb.pace_k, pace_slack);
        return hipGetLastError();
    }
    switch (look) {
    case 42: if (tall) SM_GCB(15, 4, 2); else SM_GCB(14, 4, 2); break;
    case 63: if (tall) SM_GCB(15, 6, 3); else SM_GCB(14, 6, 3); break;
    case 84: if (tall) SM_GCB(15, 8, 4); else SM_GCB(14, 8, 4); break;
    default: if (tall) SM_GCB(15, 6, 2); else SM_GCB(14, 6, 2); break;
    }
#undef SM_GCB
    return hipGetLastError();
}

}  // namespace smamd
