// xband_dev.h -- device helpers shared by the band kernels (kernels_xband.hip,
// kernels_band2.hip): range-checked buffer descriptors, vmcnt waits and the slab
// hand-off of a row block's partial sums.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

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
constexpr int kAuxSc1 = 16; // write-through store / L1-bypassing load (cross-CU hand-off)
#ifndef SM_COMBINE_SKIP_OWN
#define SM_COMBINE_SKIP_OWN 0   // 1: no load for the own slab's part (A/B: no measurable gain)
#endif

// vmcnt retires in issue order: waiting until only the N most recent vector loads
// are outstanding retires every older one, including LDS-DMA that hipcc does not count.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---------------------------------------------------------------------------
// Slab hand-off: the S tiles of one row block (one per slab of column bands)
// hold partial sums of the same rows in LDS; y = P_0 + P_1 + ... + P_{S-1} per
// row, added in slab order (P_0 starts from beta*y), the same sum whoever adds.
//
// Distributed combine: the block's rows are cut in S parts and tile s adds part s
// itself -- its own P_s straight from LDS, the other slabs' sums from memory -- so
// the tail after the slowest tile is one part (R/S rows, S-1 partial reads) per
// tile instead of all R rows by the last tile.  A tile only waits for its siblings
// when every one of them has started (ctl.started == S: they are resident and
// reach their hand-off without waiting on anything), so the wait cannot deadlock
// on a chip shared with other kernels; a tile that saw a sibling not yet started
// publishes everything and leaves its part to the last arriver (the old
// last-tile-combines-all hand-off).
//
// Control words per row block (int32 x 4, zero between launches):
//   [0] started  tiles that have begun (one agent-scope add at kernel entry)
//   [1] arrive   low 8 bits: tiles that published (S <= 64); bit 8+s: tile s combines
//                part s (S <= 16; more slabs: the last arriver combines all)
//   [2] done     tiles finished; the last one zeroes [0..2] for the next launch
// Publication follows MI355X_MICROARCH.md "Valid forms", row 1: every sum stored
// write-through (sc1), each storing wave drains vmcnt(0), a workgroup barrier, one
// agent-scope add; consumers poll with sc1 loads from one lane, a barrier, then
// read the sums with sc1 loads only.
constexpr int kCtlWords = 4;

__device__ __forceinline__ void handoff_started(int32_t *ctl, int32_t n_slabs) {
    if (n_slabs > 1 && threadIdx.x == 0)
        __hip_atomic_fetch_add(ctl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Rows [lo, hi) of the tile's sums (LDS) to `out` (block-relative), write-through.
template <int THREADS>
__device__ __forceinline__ void publish_rows(const float *yacc, float *out, bool vec,
                                             int32_t lo, int32_t hi, int32_t nr) {
    if (lo >= hi) return;
    const __amdgpu_buffer_rsrc_t o_src = rsrc(out, (uint64_t)nr * 4);
    const int32_t tid = threadIdx.x;
    const int32_t hv = vec ? lo + ((hi - lo) & ~3) : lo;   // lo is a multiple of 4
    for (int32_t i = lo + 4 * tid; i < hv; i += 4 * THREADS) {
        const float4 v = *reinterpret_cast<const float4 *>(&yacc[i]);
        const u32x4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z),
                         __float_as_uint(v.w)};
        __builtin_amdgcn_raw_buffer_store_b128(u, o_src, 4u * i, 0, kAuxSc1);
    }
    for (int32_t i = hv + tid; i < hi; i += THREADS)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(yacc[i]), o_src, 4u * i, 0, kAuxSc1);
}

// y[lo, hi) = P_0 + ... + P_{S-1} in slab order; P_me from LDS, the others from
// y (slab 0) and partials[s-1] with sc1 loads, up to 4 slabs' loads in flight.
template <int THREADS>
__device__ __forceinline__ void combine_rows(const float *yacc, float *y, const float *partials,
                                             int64_t ps, int32_t r0, int32_t nr, int32_t me,
                                             int32_t n_slabs, bool y_vec, int32_t lo, int32_t hi) {
    if (lo >= hi) return;
    const int32_t tid = threadIdx.x;
    const __amdgpu_buffer_rsrc_t y_src = rsrc(y + r0, (uint64_t)nr * 4);
    auto src = [&](int32_t s) {
        return s == 0 ? y_src : rsrc(partials + (int64_t)(s - 1) * ps + r0, (uint64_t)nr * 4);
    };
    const int32_t hv = y_vec ? lo + ((hi - lo) & ~3) : lo;
    for (int32_t i = lo + 4 * tid; i < hv; i += 4 * THREADS) {
        const float4 own = *reinterpret_cast<const float4 *>(&yacc[i]);
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int32_t s0 = 0; s0 < n_slabs; s0 += 4) {
            u32x4 pv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {   // the own slab's part comes from LDS: no request
                const int32_t s = min(s0 + j, n_slabs - 1);
                const uint32_t off = (SM_COMBINE_SKIP_OWN && (s == me || s0 + j >= n_slabs)) ? 0xFFFFFFF0u
                                                                                               : 4u * (uint32_t)i;
                pv[j] = __builtin_amdgcn_raw_buffer_load_b128(src(s), off, 0, kAuxSc1);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int32_t s = s0 + j;
                if (s >= n_slabs) break;
                const float4 v = s == me ? own
                                         : make_float4(__uint_as_float(pv[j].x), __uint_as_float(pv[j].y),
                                                       __uint_as_float(pv[j].z), __uint_as_float(pv[j].w));
                if (s == 0) {
                    acc = v;
                } else {
                    acc.x = __fadd_rn(acc.x, v.x);
                    acc.y = __fadd_rn(acc.y, v.y);
                    acc.z = __fadd_rn(acc.z, v.z);
                    acc.w = __fadd_rn(acc.w, v.w);
                }
            }
        }
        *reinterpret_cast<float4 *>(y + r0 + i) = acc;
    }
    for (int32_t i = hv + tid; i < hi; i += THREADS) {
        float a = 0.f;
        for (int32_t s = 0; s < n_slabs; ++s) {
            const float v = s == me ? yacc[i]
                                    : __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(src(s), 4u * i, 0, kAuxSc1));
            a = s == 0 ? v : __fadd_rn(a, v);
        }
        y[r0 + i] = a;
    }
}

// Beta-last form (band2 / cband with several slabs): every slab tile sums from -0.0 and
// publishes into partials[s]; y[lo, hi) = (((beta*y + P_0) + P_1) + ...) + P_{S-1}, beta*y
// formed here (kernel.cc:10-29: y *= beta unless beta == 1).  y is read by plain loads: in
// this form no tile writes a y row it does not combine itself.
template <int THREADS>
__device__ __forceinline__ void combine_rows_bl(const float *yacc, float *y, const float *partials,
                                                int64_t ps, int32_t r0, int32_t nr, int32_t me,
                                                int32_t n_slabs, bool y_vec, float beta, int32_t lo,
                                                int32_t hi) {
    if (lo >= hi) return;
    const int32_t tid = threadIdx.x;
    const __amdgpu_buffer_rsrc_t y_src = rsrc(y + r0, (uint64_t)nr * 4);
    auto src = [&](int32_t s) { return rsrc(partials + (int64_t)s * ps + r0, (uint64_t)nr * 4); };
    auto bop = [&](float v) { return beta != 1.0f ? __fmul_rn(v, beta) : v; };
    const int32_t hv = y_vec ? lo + ((hi - lo) & ~3) : lo;
    for (int32_t i = lo + 4 * tid; i < hv; i += 4 * THREADS) {
        const u32x4 yu = __builtin_amdgcn_raw_buffer_load_b128(y_src, 4u * (uint32_t)i, 0, 0);
        const float4 own = *reinterpret_cast<const float4 *>(&yacc[i]);
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int32_t s0 = 0; s0 < n_slabs; s0 += 4) {
            u32x4 pv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {   // the own slab's part and slots past S: no request
                const int32_t s = min(s0 + j, n_slabs - 1);
                const uint32_t off = (s == me || s0 + j >= n_slabs) ? 0xFFFFFFF0u : 4u * (uint32_t)i;
                pv[j] = __builtin_amdgcn_raw_buffer_load_b128(src(s), off, 0, kAuxSc1);
            }
            if (s0 == 0)
                acc = make_float4(bop(__uint_as_float(yu.x)), bop(__uint_as_float(yu.y)),
                                  bop(__uint_as_float(yu.z)), bop(__uint_as_float(yu.w)));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int32_t s = s0 + j;
                if (s >= n_slabs) break;
                const float4 v = s == me ? own
                                         : make_float4(__uint_as_float(pv[j].x), __uint_as_float(pv[j].y),
                                                       __uint_as_float(pv[j].z), __uint_as_float(pv[j].w));
                acc.x = __fadd_rn(acc.x, v.x);
                acc.y = __fadd_rn(acc.y, v.y);
                acc.z = __fadd_rn(acc.z, v.z);
                acc.w = __fadd_rn(acc.w, v.w);
            }
        }
        *reinterpret_cast<float4 *>(y + r0 + i) = acc;
    }
    for (int32_t i = hv + tid; i < hi; i += THREADS) {
        float a = bop(y[r0 + i]);
        for (int32_t s = 0; s < n_slabs; ++s) {
            const float v = s == me ? yacc[i]
                                    : __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(src(s), 4u * i, 0, kAuxSc1));
            a = __fadd_rn(a, v);
        }
        y[r0 + i] = a;
    }
}

template <int THREADS>
__device__ void slab_handoff(const float *yacc, int32_t *ctl, int32_t *s_word, float *y,
                             float *partials, int32_t n_rows, int32_t r0, int32_t nr,
                             int32_t slab, int32_t n_slabs, bool y_vec) {
    const int32_t tid = threadIdx.x;
    const int64_t ps = ((int64_t)n_rows + 3) & ~(int64_t)3;   // 16-byte aligned partial rows
    float *outp = slab == 0 ? y + r0 : partials + (int64_t)(slab - 1) * ps;
    outp = slab == 0 ? outp : outp + r0;
    const bool vec_out = slab != 0 || y_vec;
    const int32_t part = ((nr + n_slabs - 1) / n_slabs + 3) & ~3;
    auto part_lo = [&](int32_t s) { return min(s * part, nr); };
    auto part_hi = [&](int32_t s) { return min((s + 1) * part, nr); };
    if (tid == 0)   // commit bits 8..23: up to 16 slabs combine their own parts
        s_word[0] = n_slabs <= 16 &&
                    __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= n_slabs;
    __syncthreads();
    const bool committed = s_word[0] != 0;
    if (committed) {   // the own part stays in LDS
        publish_rows<THREADS>(yacc, outp, vec_out, 0, part_lo(slab), nr);
        publish_rows<THREADS>(yacc, outp, vec_out, part_hi(slab), nr, nr);
    } else {
        publish_rows<THREADS>(yacc, outp, vec_out, 0, nr, nr);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const int32_t add = 1 + (committed ? (1 << (8 + slab)) : 0);
        s_word[1] = __hip_atomic_fetch_add(ctl + 1, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + add;
        if (committed) {   // every sibling is resident: wait for all of them to publish
            int32_t a = s_word[1];
            while ((a & 0xFF) < n_slabs) {
                __builtin_amdgcn_s_sleep(2);
                a = __hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            s_word[2] = a;
        }
    }
    __syncthreads();
    const int32_t arrived = s_word[1];
    if (committed)
        combine_rows<THREADS>(yacc, y, partials, ps, r0, nr, slab, n_slabs, y_vec, part_lo(slab),
                              part_hi(slab));
    if ((arrived & 0xFF) == n_slabs) {
        // Last arriver: the parts of tiles that did not commit (their words are final:
        // every commit bit was set by the add that also counted the arrival).
        const int32_t mask = (committed ? s_word[2] : arrived) >> 8;
        for (int32_t q = 0; q < n_slabs; ++q)
            if (!((mask >> q) & 1))
                combine_rows<THREADS>(yacc, y, partials, ps, r0, nr, slab, n_slabs, y_vec,
                                      part_lo(q), part_hi(q));
    }
    if (tid == 0) {
        const int32_t d = __hip_atomic_fetch_add(ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == n_slabs - 1) {   // every tile of the block is past its last read of ctl
            __hip_atomic_store(ctl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ctl + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ctl + 2, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ---------------------------------------------------------------------------
// Epoch hand-off (the band2 / cband kernels): the same distributed combine, but the control
// words are never reset at the end of a launch, so no tile waits for a final "done" round
// trip, and the commit check is a snapshot read early in the tile (its round trip hidden
// behind the band loop) instead of a load at the start of the epilogue.
//   [0..1] started  a 64-bit monotonic count; each tile adds 1 at entry and keeps the old
//                value: its launch's generation is g = old / S (launches on one matrix are
//                ordered -- stream order or the matrix's scratch event -- so every tile of a
//                launch draws from [g S, g S + S)).  64 bits because g must be the same for
//                every tile of a launch: a 32-bit count wraps after 2^32 / S launches, and
//                where S does not divide 2^32 the launch across the wrap saw two different
//                generations and hung.  2^64 / S launches of ~30 us are ~10^6 years.
//   [2 + (g & 1)] arrive  for generation g as `arrive` above (count | commit bits); the
//                slab-0 tile zeroes the other parity's word as it leaves -- its last user
//                (launch g - 1) is complete, its next (launch g + 1) comes after this one.
// A tile commits (waits for its siblings and combines its own part) when its snapshot of
// started, read after the tile's prologue, shows all S tiles of generation g.
__device__ __forceinline__ uint64_t handoff_begin(int32_t *ctl, int32_t n_slabs) {
    if (n_slabs <= 1 || threadIdx.x != 0) return 0u;
    return __hip_atomic_fetch_add(reinterpret_cast<uint64_t *>(ctl), (uint64_t)1, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t handoff_snapshot(const int32_t *ctl, int32_t n_slabs) {
    if (n_slabs <= 1) return 0u;
    return __hip_atomic_load(reinterpret_cast<const uint64_t *>(ctl), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int THREADS, bool BL>
__device__ __forceinline__ void slab_handoff_epoch(const float *yacc, int32_t *ctl, int32_t *s_word, float *y,
                                   float *partials, int32_t n_rows, int32_t r0, int32_t nr,
                                   int32_t slab, int32_t n_slabs, bool y_vec, uint64_t old_started,
                                   uint64_t snapshot, float beta, unsigned long long *ts) {
    const int32_t tid = threadIdx.x;
    const int64_t ps = ((int64_t)n_rows + 3) & ~(int64_t)3;   // 16-byte aligned partial rows
    // BL: every slab publishes into partials[slab]; otherwise slab 0 into y, s >= 1 into partials[s-1].
    float *outp = (BL || slab != 0) ? partials + (int64_t)(BL ? slab : slab - 1) * ps + r0 : y + r0;
    const bool vec_out = BL || slab != 0 || y_vec;
    const int32_t part = ((nr + n_slabs - 1) / n_slabs + 3) & ~3;
    auto part_lo = [&](int32_t s) { return min(s * part, nr); };
    auto part_hi = [&](int32_t s) { return min((s + 1) * part, nr); };
    auto combine = [&](int32_t q) {
        if constexpr (BL)
            combine_rows_bl<THREADS>(yacc, y, partials, ps, r0, nr, slab, n_slabs, y_vec, beta, part_lo(q),
                                     part_hi(q));
        else
            combine_rows<THREADS>(yacc, y, partials, ps, r0, nr, slab, n_slabs, y_vec, part_lo(q), part_hi(q));
    };
    // Development timeline (ts != nullptr, thread 0): [0] published and drained, [1] arrival
    // add returned, [2] every sibling seen, [3] combine stores drained.
    auto stamp = [&](int k) {
        if (ts != nullptr && tid == 0) ts[k] = wall_clock64();
    };
    const uint64_t S = (uint64_t)n_slabs;
    if (tid == 0) {   // thread 0 holds the generation (handoff_begin)
        const uint64_t g = old_started / S;
        s_word[0] = n_slabs <= 16 && snapshot - g * S >= S;   // every sibling had started
        s_word[3] = (int32_t)(g & 1u);
    }
    __syncthreads();
    const bool committed = s_word[0] != 0;
    const uint32_t g = (uint32_t)s_word[3];   // the generation's parity
    int32_t *arrive = ctl + 2 + g;
    if (committed) {   // the own part stays in LDS
        publish_rows<THREADS>(yacc, outp, vec_out, 0, part_lo(slab), nr);
        publish_rows<THREADS>(yacc, outp, vec_out, part_hi(slab), nr, nr);
    } else {
        publish_rows<THREADS>(yacc, outp, vec_out, 0, nr, nr);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(0);
    if (tid == 0) {
        const int32_t add = 1 + (committed ? (1 << (8 + slab)) : 0);
        s_word[1] = __hip_atomic_fetch_add(arrive, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + add;
        stamp(1);
        if (committed) {   // every sibling is resident: wait for all of them to publish
            int32_t a = s_word[1];
            while ((a & 0xFF) < n_slabs) {
                __builtin_amdgcn_s_sleep(2);
                a = __hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            s_word[2] = a;
        }
        stamp(2);
    }
    __syncthreads();
    const int32_t arrived = s_word[1];
    if (committed) combine(slab);
    if ((arrived & 0xFF) == n_slabs) {
        // Last arriver: the parts of tiles that did not commit.
        const int32_t mask = (committed ? s_word[2] : arrived) >> 8;
        for (int32_t q = 0; q < n_slabs; ++q)
            if (!((mask >> q) & 1)) combine(q);
    }
    if (tid == 0 && slab == 0)   // the next launch's word (see above)
        __hip_atomic_store(ctl + 2 + (g ^ 1u), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ts != nullptr) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        stamp(3);
    }
}

}  // namespace
}  // namespace smamd
