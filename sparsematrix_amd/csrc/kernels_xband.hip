// kernels_xband.hip -- SpMV with x staged through LDS, one column band at a time.
//
// One workgroup (1024 threads, 16 waves) per tile = (block of rows, slab of
// column bands), one workgroup per CU.  LDS: two x bands (double-buffered) and
// the block's accumulators.  Software pipeline, one barrier per band: while
// band p is applied from one buffer, slice p+1 (held in registers since two
// bands earlier, wide float4 loads) is written to the other while slice p+3
// and the entries of band p+3 are in flight.  Each wave takes whole 64-entry
// chunks: term = x_lds[col] * (v * alpha), then the chunk's terms are added to
// the LDS accumulators in rank rounds (no two lanes touch one row in a round;
// no atomics).  Inside a tile a row's terms are therefore added in ascending
// column order (bands ascend, ranks ascend inside a band).
//
// Slab 0 starts from beta*y and writes y; slab s > 0 starts from -0.0 (the exact
// identity of fp32 addition: a row without terms in the slab keeps the sign of a
// zero y) and writes partials[s-1].  The last tile of a row block to finish (a ticket counter per
// block) adds the partials to y in slab order -- the same sum whichever tile
// finishes last.  The hand-off crosses CUs and XCDs: the slab sums are stored
// write-through (sc1) and drained before the ticket, and the last tile reads
// every one of them with sc1 loads (cdna_hip_programming.md §6 Guideline 16).
// With one slab (the "exact" layout) every row is summed exactly in the
// reference's order: bit-identical.  Layout and builder: xband.h / xband.cpp.
//
// Why x goes through LDS (profiles/r01_microbench.txt): random 4-byte gathers
// are TA-bound (~0.6 lanes/clk/CU); wide loads of a band are not.  The cost is
// that every tile sweeps its slab of x: blocked tiles (16K rows) sweep 4x less
// x per CU than exact ones (4K rows) -- the x sweep, L2 -> CU at ~85 GB/s per
// CU, is what bounds the exact layout.
#include "sm_internal.h"
#include "xband.h"
#include "xband_dev.h"

#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace smamd {
namespace {

// SM_XBAND_DMA=0: blocked x slices through a 4-slice register ring instead of LDS-DMA;
// SM_XBAND_LOADERS=0/4/8: waves that only stage x (0: every wave stages and applies).  Both for A/B comparisons; read once.
bool xband_dma_setting() {
    static const bool on = [] {
        const char *e = dev_env("SM_XBAND_DMA");
        return !(e && atoi(e) == 0);
    }();
    return on;
}
int xband_loaders_setting() {   // SM_XBAND_LOADERS = 0 (default), 4 or 8 loader waves
    static const int n = [] {
        const char *e = dev_env("SM_XBAND_LOADERS");
        const int v = e ? atoi(e) : 0;
        return v == 4 || v == 8 ? v : 0;
    }();
    return n;
}

// One asm statement naming every value: all of them are materialised (one
// s_waitcnt) before anything after it, so hipcc cannot sink a read below a later
// write it might alias (it would re-read after that write: one LDS round trip per
// chunk instead of one per band).
template <int N>
__device__ __forceinline__ void pin_all(float *a, float *b) {
    if constexpr (N == 1) {
        asm volatile("" : "+v"(a[0]), "+v"(b[0]));
    } else if constexpr (N == 2) {
        asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(b[0]), "+v"(b[1]));
    } else if constexpr (N == 3) {
        asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]));
    } else if constexpr (N == 4) {
        asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]),
                     "+v"(b[2]), "+v"(b[3]));
    } else {
        static_assert(N == 5, "CAP of 1 to 5");
        asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(b[0]),
                     "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]));
    }
}

// ABL (ablation, development only, SM_XBAND_ABLATE): bit 1 skips the apply, bit 2
// the x slice loads, bit 4 the entry loads, bit 16 the per-band barrier; the staged
// slices are kept live so nothing upstream is dead-code removed; bit 128 skips the
// slice stores into LDS (the loaded values kept live), 256 the whole band loop, 512
// the slab hand-off and combine (plain stores instead), 2048 everything (launch cost), 4096 the
// value loads (word loads kept: half the entry bytes).  Bit 32 records
// s_memtime stamps (tile 0, 6 per band per wave, bands < 32) into y[0, 3072).
// Timing only: results are wrong.
// XR: x slices held in registers (2 or 4): slice p+XR+(XR==2) is loaded at band p and
// stored XR-1+(XR==2) bands later -- a deeper ring hides more L2 latency per band.
// XR == 0: no register ring -- slices go HBM/L2 -> LDS directly (LDS-DMA) into a
// ring of three LDS buffers, slice p+2 issued at band p.
// PRIO: wave priority (s_setprio) while a wave applies a band -- its LDS reads and
// writes then win the issue arbitration over the other waves' load issue, which the
// band's barrier waits for anyway: 45.4-46.3 vs 47.0 us on config 2.
// SM_XBAND_PRIO=0..3 overrides (A/B).
template <int THREADS, int BAND_LOG2, int ROWS_LOG2, int CAP, int XR, int ABL = 0,
          bool STAGGER = true, int LOADERS = 0, int PRIO = 2>
__global__ __launch_bounds__(THREADS) void spmv_xband_kernel(
    int32_t n_rows, int32_t n_cols, int32_t block_rows, int32_t n_bands, int32_t n_slabs,
    int32_t slab_bands, const int32_t *__restrict__ chunk_start,
    const uint32_t *__restrict__ word, const float *__restrict__ val,
    const float *__restrict__ x, float *__restrict__ y, float *__restrict__ partials,
    int32_t *__restrict__ tickets, float alpha, float beta) {
    constexpr int BAND = 1 << BAND_LOG2;
    constexpr int BROWS = 1 << ROWS_LOG2;
    constexpr XbBits kBits = xb_bits(BAND_LOG2, ROWS_LOG2);
    constexpr uint32_t kColMask = (1u << kBits.col) - 1u;
    constexpr uint32_t kRankMask = (1u << kBits.rank) - 1u;
    constexpr uint32_t kDummyRank = kBits.dummy_rank();
    constexpr uint32_t kDummyWord = kBits.dummy_word();
    constexpr int kWaves = THREADS / 64;
    constexpr int kXv = BAND / (4 * THREADS);   // float4 per thread per band
    static_assert(kXv >= 1, "band too small for the workgroup");
    static_assert(XR == 0 || XR == 2 || XR == 4, "x ring of 2 or 4 slices, or LDS-DMA");
    constexpr bool kDma = XR == 0;
    constexpr int kXAhead = XR == 4 ? 4 : 3;    // register ring: slice loaded at band p: p + kXAhead
    // LDS: x buffers (three for LDS-DMA when they fit: two bands of lookahead),
    // then per-lane scratch write slots when they fit too.
    constexpr int kLds = 163840 / (1024 / THREADS);   // LDS per CU / workgroups per CU
    constexpr int kXBufs = kDma && 3 * BAND * 4 + BROWS * 4 <= kLds ? 3 : 2;
    constexpr int kScratch = kXBufs * BAND * 4 + (BROWS + 64) * 4 <= kLds ? 64 : 0;
    constexpr int kDmaAhead = kXBufs - 1;       // LDS-DMA: slice p + kDmaAhead issued at band p
    // vmcnt at the end of band p that retires slice p+1 (issued kDmaAhead-1 bands
    // earlier, each band issuing its slice then its entries: 2*CAP loads).
    constexpr int kDmaWait = kDmaAhead == 2 ? 4 * CAP + kXv : 2 * CAP;
    // LOADERS (LDS-DMA only, SM_XBAND_LOADERS=4|8, measured alternative): the last
    // kLoaders waves only stage x (kPerLoader LDS-DMA pieces each per band, then a
    // wait that retires nothing but x); the other kComp waves only load entries and
    // apply.  Motivation: vmcnt retires in issue order, so a wave with entry loads in
    // flight that waits for its x pieces also waits for every older entry load.
    // Measured 49.2 us (4 or 8 loaders) vs 46.5 us without: a wave issues one 1 KiB
    // LDS-DMA piece per ~150-190 cycles, so few loader waves serialise the x staging
    // that 16 waves issue in parallel.  Default: 0 (every wave
    // stages its share of x and applies).
    constexpr bool kRoles = LOADERS > 0 && kDma;
    constexpr int kLoaders = kRoles ? LOADERS : 0;
    constexpr int kComp = kWaves - kLoaders;
    constexpr int kPieces = BAND / 256;                 // 1 KiB LDS-DMA pieces per slice
    constexpr int kPerLoader = kRoles ? kPieces / kLoaders : 1;
    static_assert(!kRoles || (kPieces % (kRoles ? kLoaders : 1) == 0 && kXBufs == 3),
                  "loader split");
    __shared__ __attribute__((aligned(16))) float xs[kXBufs][BAND];
    __shared__ float yacc[BROWS + kScratch];   // + one scratch slot per lane (writes that land nowhere)
    if (ABL & 2048) return;   // launch cost only
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int32_t b = blockIdx.x / n_slabs;
    const int32_t slab = blockIdx.x - b * n_slabs;
    const int32_t p_first = slab * slab_bands;
    const int32_t nb = min(slab_bands, n_bands - p_first);   // bands of this tile (>= 1)
    // (not in the tracing build: tile 0 returns early and never arrives)
    if (!(ABL & (512 | 32))) handoff_started(tickets + (int64_t)b * kCtlWords, n_slabs);
    const int32_t r0 = b * block_rows;
    const int32_t nr = min(block_rows, n_rows - r0);
    const int32_t *csg = chunk_start + (int64_t)b * n_bands + p_first;
    const int32_t c_first = csg[0];
    const int32_t c_last = csg[nb];
    const int64_t x0 = (int64_t)p_first * BAND;
    const __amdgpu_buffer_rsrc_t xr_src = rsrc(x + x0, (uint64_t)(n_cols - x0) * 4);
    const __amdgpu_buffer_rsrc_t w_src =
        rsrc(word + (int64_t)c_first * 64, (uint64_t)(c_last - c_first) * 256);
    const __amdgpu_buffer_rsrc_t v_src =
        rsrc(val + (int64_t)c_first * 64, (uint64_t)(c_last - c_first) * 256);
    // Chunk table window in registers: lane l holds cs[cw + l] (lo) and
    // cs[cw + 64 + l] (hi), tile-relative; read by readlane with a branch-free
    // select.  Every 64 bands the window advances: hi (loaded 64 bands earlier)
    // becomes lo and the next hi is prefetched -- no load is waited for at once.
    // The raw table values are kept (c_first is subtracted after the readlane), so
    // the prefetched hi half is not touched -- and not waited for -- until it
    // becomes lo 64 bands later.
    int32_t cw = 0;
    int32_t cs_lo = csg[min(lane, nb)];
    int32_t cs_hi = csg[min(64 + lane, nb)];
    auto advance_cs_window = [&]() {
        cw += 64;
        cs_lo = cs_hi;
        cs_hi = csg[min(cw + 64 + lane, nb)];
    };
    auto cs_at = [&](int32_t i) -> int32_t {   // i in [cw, cw + 128), wave-uniform
        const int32_t j = i - cw;
        const int32_t lo = __builtin_amdgcn_readlane(cs_lo, j & 63);
        const int32_t hi = __builtin_amdgcn_readlane(cs_hi, j & 63);
        return (j < 64 ? lo : hi) - c_first;
    };

    auto load_slice = [&](int32_t p, float4 *xr) {
#pragma unroll
        for (int k = 0; k < kXv; ++k) {
            const uint32_t off = p < nb ? 4u * (uint32_t)(p * BAND + 4 * (tid + k * THREADS))
                                        : 0xFFFFFFF0u;
            u32x4 v = {off, off, off, off};
            if (!(ABL & 2)) v = __builtin_amdgcn_raw_buffer_load_b128(xr_src, off, 0, 0);
            xr[k] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y),
                                __uint_as_float(v.z), __uint_as_float(v.w));
        }
    };
    auto store_slice = [&](int buf, const float4 *xr) {
#pragma unroll
        for (int k = 0; k < kXv; ++k) {
            if (ABL & 128)
                asm volatile("" ::"v"(xr[k].x), "v"(xr[k].y), "v"(xr[k].z), "v"(xr[k].w));
            else
                *reinterpret_cast<float4 *>(&xs[buf][4 * (tid + k * THREADS)]) = xr[k];
        }
    };
    // LDS-DMA of slice p into buffer `buf`: piece m (256 floats, 1 KiB) is
    // wave-instruction k of wave m % 16.  Issued from asm so hipcc does not count
    // it (a counted LDS-DMA makes hipcc drain vmcnt at every barrier and at every
    // use of an ordinary load); wait_vmcnt retires it before the barrier.
    const uint32_t xs_lds = (uint32_t)(size_t)(__attribute__((address_space(3))) float *)&xs[0][0];
    auto dma_slice = [&](int32_t p, int buf) {
#pragma unroll
        for (int k = 0; k < kXv; ++k) {
            const int m = k * (THREADS / 64) + wave;
            const uint32_t voff = p < nb && !(ABL & 2)
                                      ? 4u * (uint32_t)(p * BAND + m * 256 + lane * 4)
                                      : 0xFFFFFFF0u;
            const uint32_t lds =
                __builtin_amdgcn_readfirstlane(xs_lds + 4u * (uint32_t)(buf * BAND + m * 256));
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(voff), "s"(xr_src), "s"(lds)
                : "memory");
        }
    };
    // LOADERS: loader li = wave - kComp stages pieces li, li + kLoaders, ... of slice p.
    auto dma_slice_loader = [&](int32_t p, int buf) {
        const int li = wave - kComp;
#pragma unroll
        for (int k = 0; k < kPerLoader; ++k) {
            const int m = k * kLoaders + li;
            const uint32_t voff =
                p < nb ? 4u * (uint32_t)(p * BAND + m * 256 + lane * 4) : 0xFFFFFFF0u;
            const uint32_t lds =
                __builtin_amdgcn_readfirstlane(xs_lds + 4u * (uint32_t)(buf * BAND + m * 256));
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(voff), "s"(xr_src), "s"(lds)
                : "memory");
        }
    };
    // Chunk c of band p for this wave.  A slot beyond the band's last chunk
    // loads from past the descriptor's range (no memory request, reads 0): words
    // are stored XOR the dummy word, so it is a dummy entry without a select
    // (a select right after the load makes hipcc wait for it there -- at the
    // loop's back edge -- instead of three bands later at the use).
    auto load_entries = [&](int32_t p, uint32_t *w, float *v) {
        const bool inb = p < nb;
        const int32_t c0 = inb ? cs_at(p) : 0;
        const int32_t c1 = inb ? cs_at(p + 1) : 0;
#pragma unroll
        for (int k = 0; k < CAP; ++k) {
            const int32_t c = c0 + wave + k * kComp;
            const uint32_t off = c < c1 ? 4u * (uint32_t)(c * 64 + lane) : 0xFFFFFF00u;
            uint32_t wl = ((uint32_t)(lane * 131) & kColMask) ^ kDummyWord, vl = off;
            if (!(ABL & 4)) {
                wl = __builtin_amdgcn_raw_buffer_load_b32(w_src, off, 0, kAuxNt);
                if (!(ABL & 4096)) vl = __builtin_amdgcn_raw_buffer_load_b32(v_src, off, 0, kAuxNt);
            }
            w[k] = wl;
            v[k] = __uint_as_float(vl);
        }
    };
    // All chunks of a band at once: every lane's x and accumulator reads issue
    // together (one LDS wait).  A row's terms inside a band form one segment of
    // consecutive lanes of one chunk (ranks 0, 1, ...); the segment's running sum
    // moves up the lanes in registers (DPP wave_shr:1, one round per rank) and
    // only its last lane writes the accumulator -- the terms still added one at a
    // time in ascending column order.  Chunks of a band, in this wave and in every
    // other wave, touch disjoint rows.
    auto shr1 = [](float v) {   // lane i <- lane i-1 (lane 0 never has rank >= 1)
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, false));
    };
    auto shl1 = [](uint32_t v) {   // lane i <- lane i+1; lane 63 <- the dummy rank
        return (uint32_t)__builtin_amdgcn_update_dpp((int)kDummyRank, (int)v, 0x130, 0xF, 0xF, false);
    };
    auto apply_band = [&](const float *xb, const uint32_t *wa, const float *va) {
        if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(PRIO);
        float xv[CAP], yv[CAP];
        uint32_t rk[CAP], rl[CAP];
        bool live[CAP];
        bool more = false;
#pragma unroll
        for (int k = 0; k < CAP; ++k) {
            const uint32_t wd = wa[k] ^ kDummyWord;
            rk[k] = (wd >> kBits.col) & kRankMask;
            live[k] = rk[k] != kDummyRank;
            rl[k] = wd >> (kBits.col + kBits.rank);   // dummies decode to row 0, column 0
            xv[k] = xb[wd & kColMask];
            yv[k] = yacc[rl[k]];
            more |= live[k] && rk[k] > 0;
        }
        pin_all<CAP>(xv, yv);
        float t[CAP], acc[CAP];
#pragma unroll
        for (int k = 0; k < CAP; ++k) {
            t[k] = __fmul_rn(xv[k], __fmul_rn(va[k], alpha));
            acc[k] = __fadd_rn(yv[k], t[k]);
        }
        if (__any(more)) {
            for (uint32_t r = 1;; ++r) {
                bool again = false;
#pragma unroll
                for (int k = 0; k < CAP; ++k) {
                    const float prev = shr1(acc[k]);
                    if (rk[k] == r) acc[k] = __fadd_rn(prev, t[k]);
                    again |= live[k] && rk[k] > r;
                }
                if (!__any(again)) break;
            }
        }
#pragma unroll
        for (int k = 0; k < CAP; ++k) {   // every lane writes: the segment's last to its row
            const bool last = live[k] && shl1(rk[k]) != rk[k] + 1u;
            if constexpr (kScratch > 0)
                yacc[last ? rl[k] : (uint32_t)(BROWS + lane)] = acc[k];
            else if (last)
                yacc[rl[k]] = acc[k];
        }
        if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(0);
    };

    // Register rings with static roles (the band loop is unrolled by kER, so every
    // ring index is a compile-time constant and no register ever moves -- a move
    // would make hipcc wait for the load that filled it): x slice q lives in
    // X[q % XR], the entries of band q in W/V[q % kER], loaded kEAhead bands early.
    constexpr int kEAhead = 3;                  // entries' lookahead (5 measured: no gain)
    constexpr int kER = kEAhead > 3 ? 8 : 4;    // entry ring = loop unroll
    constexpr int kXR = XR > 0 ? XR : 1;
    static_assert(kER % kXR == 0 && kEAhead < kER, "ring sizes");
    float4 X[kXR][kXv];
    uint32_t W[kER][CAP];
    float V[kER][CAP];
    // Accumulators first: this loop's own loads are drained before the pipeline
    // starts.  Then the prologue issues its loads in exactly the order the loop
    // leaves them pending at its back edge, so hipcc's vmcnt bookkeeping merges
    // the two paths into the loop header without falling back to tighter waits.
    // All of a thread's rows in flight at once (one 16-byte load per 4 rows when y
    // is aligned, else one dword load per row; rows past nr read 0 and are never
    // written back): a load-then-store loop would pay one memory latency per row.
    constexpr int kQ = BROWS / (4 * THREADS);   // float4 rows per thread
    const bool y_vec = ((uintptr_t)(y + r0) & 15) == 0;
    if (slab == 0) {
        const __amdgpu_buffer_rsrc_t yi_src = rsrc(y + r0, (uint64_t)nr * 4);
        float4 v[kQ];
        if (y_vec) {
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(
                    yi_src, 16u * (uint32_t)(tid + q * THREADS), 0, 0);
                v[q] = make_float4(__uint_as_float(u.x), __uint_as_float(u.y),
                                   __uint_as_float(u.z), __uint_as_float(u.w));
            }
        } else {
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                const uint32_t o = 16u * (uint32_t)(tid + q * THREADS);
                v[q] = make_float4(
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o, 0, 0)),
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 4, 0, 0)),
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 8, 0, 0)),
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 12, 0, 0)));
            }
        }
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            if (beta != 1.0f)
                v[q] = make_float4(__fmul_rn(v[q].x, beta), __fmul_rn(v[q].y, beta),
                                   __fmul_rn(v[q].z, beta), __fmul_rn(v[q].w, beta));
            *reinterpret_cast<float4 *>(&yacc[4 * (tid + q * THREADS)]) = v[q];
        }
    } else {
#pragma unroll
        for (int q = 0; q < kQ; ++q)
            *reinterpret_cast<float4 *>(&yacc[4 * (tid + q * THREADS)]) = make_float4(-0.f, -0.f, -0.f, -0.f);
    }
    if constexpr (kRoles) {
        // Loaders: slices 0 and 1 in flight, slice 0 landed; then per band: slice
        // p+2 into the buffer band p-1 freed, wait until only those pieces fly (slice
        // p+1 landed), barrier.  Compute waves: entries 0..2 in flight; per band:
        // entries p+3, apply band p, barrier.  One barrier per band in both roles.
        const int32_t nbr = (ABL & 256) ? 0 : (nb + kER - 1) / kER * kER;
        const bool rtrace = (ABL & 32) && blockIdx.x == 0;   // stamps (development only)
        auto rstamp = [&](int32_t p, int k) {
            if (!rtrace || p >= 32) return;
            const uint64_t t = __builtin_amdgcn_s_memtime();
            if (lane == 0) reinterpret_cast<uint32_t *>(y)[wave * 192 + p * 6 + k] = (uint32_t)t;
        };
        if (wave >= kComp) {
            dma_slice_loader(0, 0);
            dma_slice_loader(1, 1);
            wait_vmcnt<kPerLoader>();
            __syncthreads();
            for (int32_t p = 0; p < nbr; ++p) {
                rstamp(p, 0);
                dma_slice_loader(p + 2, (p + 2) % kXBufs);
                rstamp(p, 1);
                rstamp(p, 2);
                wait_vmcnt<kPerLoader>();
                rstamp(p, 3);
                rstamp(p, 4);
                __syncthreads();
                rstamp(p, 5);
            }
        } else {
#pragma unroll
            for (int q = 0; q < kEAhead; ++q) load_entries(q, W[q], V[q]);
            __syncthreads();
            for (int32_t p = 0; p < nbr; p += kER) {
#pragma unroll
                for (int u = 0; u < kER; ++u) {
                    rstamp(p + u, 0);
                    if (p + u + kEAhead >= cw + 64) advance_cs_window();
                    rstamp(p + u, 1);
                    load_entries(p + u + kEAhead, W[(u + kEAhead) % kER], V[(u + kEAhead) % kER]);
                    rstamp(p + u, 2);
                    if (rtrace) {
#pragma unroll
                        for (int k = 0; k < CAP; ++k) asm volatile("" ::"v"(W[u][k]), "v"(V[u][k]));
                    }
                    rstamp(p + u, 3);
                    apply_band(xs[(p + u) % kXBufs], W[u], V[u]);
                    rstamp(p + u, 4);
                    __syncthreads();
                    rstamp(p + u, 5);
                }
            }
        }
    } else {
        // Prologue: the loads the loop expects in flight, issued in its order
        // (per band q: slice q+kDmaAhead, then entries q+kEAhead).
        if constexpr (kDma && kDmaAhead == 2) {   // pending after: E(A-2) D1 E(A-1)
    #pragma unroll
            for (int q = 0; q <= kEAhead - 3; ++q) load_entries(q, W[q], V[q]);
            dma_slice(0, 0);
            load_entries(kEAhead - 2, W[kEAhead - 2], V[kEAhead - 2]);
            dma_slice(1, 1);
            load_entries(kEAhead - 1, W[kEAhead - 1], V[kEAhead - 1]);
            wait_vmcnt<kDmaWait>();   // slice 0 landed
        } else if constexpr (kDma) {              // pending after: E(A-1)
    #pragma unroll
            for (int q = 0; q <= kEAhead - 2; ++q) load_entries(q, W[q], V[q]);
            dma_slice(0, 0);
            load_entries(kEAhead - 1, W[kEAhead - 1], V[kEAhead - 1]);
            wait_vmcnt<kDmaWait>();   // slice 0 landed
        } else if constexpr (XR == 4) {   // pending after: X1 E0 X2 E1 X3 E2
            load_slice(0, X[0]);
            load_slice(1, X[1]);
            load_entries(0, W[0], V[0]);
            load_slice(2, X[2 % kXR]);
            load_entries(1, W[1], V[1]);
            load_slice(3, X[3 % kXR]);
            load_entries(2, W[2], V[2]);
            store_slice(0, X[0]);
        } else {                   // pending after: E0 X1 E1 X0 E2
            load_slice(0, X[0]);
            load_entries(0, W[0], V[0]);
            load_slice(1, X[1 % kXR]);
            load_entries(1, W[1], V[1]);
            store_slice(0, X[0]);
            load_slice(2, X[0]);
            load_entries(2, W[2], V[2]);
        }
        __syncthreads();

        // Band p (register staging): buffer p&1 holds slice p (visible); the ring holds
        // slice p+1.  One barrier per band: the stores of slice p+1 into buffer (p+1)&1
        // (freed by the previous barrier) and this band's reads of buffer p&1 both
        // finish before it.  Slice p+kXAhead goes to the ring slot freed last (XR == 4:
        // slice p's, stored a band ago; XR == 2: slice p+1's, stored just now).  LDS-DMA:
        // slice p+kDmaAhead goes straight into the buffer freed by the last barrier.
        // Entries of band p+kEAhead reuse the set of band p+kEAhead-kER.  Loads past the
        // tile's last band are sent past the descriptors' ranges and never applied.
        const bool tracing = (ABL & 32) && blockIdx.x == 0;
        auto stamp = [&](int32_t p, int k) {
            if (!tracing || p >= 32) return;
            const uint64_t t = __builtin_amdgcn_s_memtime();
            if (lane == 0) reinterpret_cast<uint32_t *>(y)[wave * 192 + p * 6 + k] = (uint32_t)t;
        };
        // LATE (waves >= kWaves/2 when STAGGER): apply first, then issue the band's
        // loads -- so one half of the waves fills the TA queue while the other half
        // works the LDS, instead of all 16 doing each in lockstep after the barrier.
        // Same issue order per band in both roles, so the vmcnt plan is unchanged.
        auto step = [&](auto late, int32_t p, float4 *xst, float4 *xld, uint32_t *wa, float *va,
                        uint32_t *wl, float *vl) {
            constexpr bool kLate = decltype(late)::value;
            stamp(p, 0);
            if (p + kEAhead >= cw + 64) advance_cs_window();   // reads cs[p+A], cs[p+A+1]
            auto issue = [&]() {
                if constexpr (kDma) {
                    // The buffer of slice p+kDmaAhead-kXBufs = p-1, freed by the last barrier.
                    dma_slice(p + kDmaAhead, (p + kDmaAhead) % kXBufs);
                    stamp(p, 1);
                } else {
                    store_slice((p + 1) & 1, xst);
                    stamp(p, 1);
                    load_slice(p + kXAhead, xld);
                }
                load_entries(p + kEAhead, wl, vl);
                stamp(p, 2);
            };
            auto work = [&]() {
                if (tracing) {
    #pragma unroll
                    for (int k = 0; k < CAP; ++k) asm volatile("" ::"v"(wa[k]), "v"(va[k]));
                    stamp(p, 3);
                }
                // Every chunk of the band is in registers: the builder guarantees at
                // most CAP chunks per wave per band (no loop of loads in the pipeline,
                // so hipcc can count vmcnt exactly).
                if (ABL & 1) {
    #pragma unroll
                    for (int k = 0; k < CAP; ++k) asm volatile("" ::"v"(wa[k]), "v"(va[k]));
                } else {
                    apply_band(xs[kDma ? p % kXBufs : p & 1], wa, va);
                }
                stamp(p, 4);
            };
            if constexpr (kLate) {
                work();
                issue();
            } else {
                issue();
                work();
            }
            if constexpr (kDma) wait_vmcnt<kDmaWait>();   // slice p+1 landed (entries may fly)
            if (!(ABL & 16)) __syncthreads();
            stamp(p, 5);
        };
        // Whole groups of kER bands, no early exit: a break out of the unrolled body
        // would share the loop latch and make hipcc's vmcnt bookkeeping merge the
        // break paths into the loop header (tight waits in the first step).  Steps
        // past the tile's last band see only dummy entries and apply nothing.
        const int32_t nbu = (ABL & 256) ? 0 : (nb + kER - 1) / kER * kER;
        auto band_loop = [&](auto late) {
            for (int32_t p = 0; p < nbu; p += kER) {
    #pragma unroll
                for (int u = 0; u < kER; ++u) {
                    // x: store slice p+u+1 from X[(u+1) % XR]; load slice p+u+kXAhead into the
                    // slot freed last (XR 4: slice p+u's; XR 2: the one just stored).
                    float4 *xst = X[(u + 1) % kXR];
                    float4 *xld = X[(XR == 4 ? u : u + 1) % kXR];
                    step(late, p + u, xst, xld, W[u], V[u], W[(u + kEAhead) % kER],
                         V[(u + kEAhead) % kER]);
                }
            }
        };
        // Two whole copies of the loop (a branch inside it would merge the two roles'
        // vmcnt states): waves 0..7 issue-then-apply, waves 8..15 apply-then-issue.
        if (STAGGER && wave >= kWaves / 2)
            band_loop(std::true_type{});
        else
            band_loop(std::false_type{});
    }
    if ((ABL & 32) && blockIdx.x == 0) return;   // stamps only
    if (n_slabs == 1 || (ABL & 512)) {
        const int32_t nv = y_vec ? (nr & ~3) : 0;   // float4 rows, then the rest
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int32_t i = 4 * (tid + q * THREADS);
            if (i < nv) *reinterpret_cast<float4 *>(y + r0 + i) = *reinterpret_cast<const float4 *>(&yacc[i]);
        }
        for (int32_t i = nv + tid; i < nr; i += THREADS) y[r0 + i] = yacc[i];
    } else {
        // LDS is full: the hand-off's broadcast words go to the x buffer, no longer
        // read -- once every LDS-DMA (the loop's past-the-end ones too) has landed.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        slab_handoff<THREADS>(yacc, tickets + (int64_t)b * kCtlWords,
                              reinterpret_cast<int32_t *>(&xs[0][0]), y, partials, n_rows, r0, nr,
                              slab, n_slabs, y_vec);
    }
    if (ABL && beta == -12345.0f) y[tid] = xs[0][tid] + xs[1][tid];   // keep the staging live
}

template <int THREADS, int BAND_LOG2, int ROWS_LOG2, int CAP, int ABL>
hipError_t launch_tiles(const XbandDev &xb, int32_t n_rows, int32_t n_cols, const float *x,
                        float *y, float alpha, float beta, int loaders, hipStream_t s) {
    // x staging: blocked (2 float4 per thread per slice) by LDS-DMA into three LDS
    // buffers, issued by 4 loader waves (roles) or by every wave; exact (4 float4
    // per slice, no room for a third 64 KiB buffer) through a 2-slice register ring.
    constexpr int XRr = (1 << BAND_LOG2) / (4 * THREADS) <= 2 ? 4 : 2;
    const bool dma = XRr == 4 && xband_dma_setting();
#define SM_XBL(XR, RL)                                                                          \
    hipLaunchKernelGGL((spmv_xband_kernel<THREADS, BAND_LOG2, ROWS_LOG2, CAP, XR, ABL, true, RL>), \
                       dim3((unsigned)((int64_t)xb.n_blocks * xb.n_slabs)), dim3(THREADS), 0, s,  \
                       n_rows, n_cols, xb.block_rows, xb.n_bands, xb.n_slabs, xb.slab_bands,     \
                       xb.d_chunk_start, xb.d_word, xb.d_val, x, y, xb.d_partials, xb.d_tickets, \
                       alpha, beta)
#ifdef SM_DEV
    // Development builds: loader-wave roles, the register ring on the blocked kind
    // (SM_XBAND_DMA=0) and the wave priority A/B (SM_XBAND_PRIO).
    if (dma) {
        if constexpr (XRr == 4) {
            if (loaders == 8)
                SM_XBL(0, 8);
            else if (loaders == 4)
                SM_XBL(0, 4);
            else if (ABL == 0 && dev_env("SM_XBAND_PRIO") && atoi(dev_env("SM_XBAND_PRIO")) != 2) {
                const int pr = atoi(dev_env("SM_XBAND_PRIO"));
#define SM_XBP(P)                                                                                 \
    hipLaunchKernelGGL((spmv_xband_kernel<THREADS, BAND_LOG2, ROWS_LOG2, CAP, 0, ABL, true, 0, P>), \
                       dim3((unsigned)((int64_t)xb.n_blocks * xb.n_slabs)), dim3(THREADS), 0, s,  \
                       n_rows, n_cols, xb.block_rows, xb.n_bands, xb.n_slabs, xb.slab_bands,     \
                       xb.d_chunk_start, xb.d_word, xb.d_val, x, y, xb.d_partials, xb.d_tickets, \
                       alpha, beta)
                if (pr == 0) SM_XBP(0); else if (pr == 1) SM_XBP(1); else SM_XBP(3);
#undef SM_XBP
            }
            else
                SM_XBL(0, 0);
        }
    } else {
        SM_XBL(XRr, 0);
    }
#else
    (void)loaders;
    (void)dma;
    if constexpr (XRr == 4) SM_XBL(0, 0);   // x by LDS-DMA
    else SM_XBL(XRr, 0);                     // exact kind: register ring
#endif
#undef SM_XBL
    return hipGetLastError();
}

template <int THREADS, int BAND_LOG2, int ROWS_LOG2>
hipError_t launch_kind(const XbandDev &xb, int32_t n_rows, int32_t n_cols, const float *x,
                       float *y, float alpha, float beta, hipStream_t s) {
#ifdef SM_DEV
    const char *abl_env = dev_env("SM_XBAND_ABLATE");   // development only: results wrong
    const int abl = abl_env ? atoi(abl_env) : 0;
#else
    constexpr int abl = 0;
#endif
    // Loader waves on the LDS-DMA path (SM_XBAND_LOADERS, development builds, default
    // none; a count whose applying waves would need more than kXbMaxCap chunks per band
    // is halved).
    constexpr bool kDmaKind = (1 << BAND_LOG2) / (4 * THREADS) <= 2;
    int loaders = kDmaKind && (abl == 0 || abl == 32) && xband_dma_setting()
                      ? xband_loaders_setting() : 0;
    auto cap_for = [&](int ld) {   // chunks per applying wave per band
        const int waves = THREADS / 64 - ld;
        return (xb.max_chunks_per_band + waves - 1) / waves;
    };
    while (loaders > 0 && cap_for(loaders) > kXbMaxCap) loaders /= 2;   // 8 -> 4 -> 2 -> 1 -> 0
    if (loaders != 8 && loaders != 4) loaders = 0;
    const int64_t cap = cap_for(loaders);
#define SM_XBT(C, A) launch_tiles<THREADS, BAND_LOG2, ROWS_LOG2, C, A>(xb, n_rows, n_cols, x, y, alpha, beta, loaders, s)
#ifdef SM_DEV
    if (abl) {
        if (cap > 4) return hipErrorInvalidValue;
        switch (abl) {
        case 1: return SM_XBT(4, 1);
        case 2: return SM_XBT(4, 2);
        case 4: return SM_XBT(4, 4);
        case 5: return SM_XBT(4, 5);
        case 16: return SM_XBT(4, 16);
        case 32: return SM_XBT(4, 32);
        case 21: return SM_XBT(4, 21);
        case 7: return SM_XBT(4, 7);
        case 256: return SM_XBT(4, 256);
        case 512: return SM_XBT(4, 512);
        case 768: return SM_XBT(4, 768);
        case 2048: return SM_XBT(4, 2048);
        case 37: return SM_XBT(4, 37);
        case 4096: return SM_XBT(4, 4096);
        case 8192: return SM_XBT(4, 8192);   // no ablation: the full kernel at CAP 4 (baseline for the others)
        case 4097: return SM_XBT(4, 4097);
        default: return hipErrorInvalidValue;
        }
    }
#endif
    if (cap <= 1) return SM_XBT(1, 0);
    if (cap <= 2) return SM_XBT(2, 0);
    if (cap <= 3) return SM_XBT(3, 0);
    if (cap <= 4) return SM_XBT(4, 0);
    if (cap <= kXbMaxCap) return SM_XBT(5, 0);
#undef SM_XBT
    return hipErrorInvalidValue;
}


// ---------------------------------------------------------------------------
// Gather-band kernel (kind kXbGather).  Same tiles, chunks,
// rank rounds, slab hand-off and summation order as the kernel above, but x is
// not staged through LDS: the builder lists a band's segments by first column,
// so the 64 x gathers of one wave-instruction fall in a window of ~1 KiB (about
// 8 lanes per 128-byte line at 16 terms per row), which the TA coalesces --
// windowed gathers run at the index-stream rate (profiles/r01_microbench.txt)
// while fully random ones are TA-bound.  Per band a wave loads the entries of
// band p+EA, gathers the x values of band p+GA (their words arrived EA-GA
// bands ago) and applies band p: only the accumulator read and write touch LDS,
// no x slice is stored and LDS holds nothing but the accumulators.  One barrier
// per band keeps a row's terms in ascending column order.  Slower than the
// LDS-staged kernel on config 2 (54 vs 48 us, DESIGN.md §3.4: the gathers and the
// apply each add ~10 us that do not overlap the entry stream) but faster on wide
// slices, where a blocked tile would sweep many MiB of x through LDS for few
// terms: AUTO takes it past 3M columns (32K-column bands; 8M: 93 vs 145 us,
// DESIGN.md §6).
template <int N>
__device__ __forceinline__ void pin_one(float *a) {
#pragma unroll
    for (int k = 0; k < N; ++k) asm volatile("" : "+v"(a[k]));
}

// ABL (development only, SM_GBAND_ABLATE; results wrong): 1 skips the x gathers,
// 2 the apply (loaded values kept live), 4 the slab hand-off (plain stores).
template <int THREADS, int BAND_LOG2, int ROWS_LOG2, int CAP, int EA, int GA, int ABL = 0>
__global__ __launch_bounds__(THREADS) void spmv_gband_kernel(
    int32_t n_rows, int32_t n_cols, int32_t block_rows, int32_t n_bands, int32_t n_slabs,
    int32_t slab_bands, const int32_t *__restrict__ chunk_start,
    const uint32_t *__restrict__ word, const float *__restrict__ val,
    const float *__restrict__ x, float *__restrict__ y, float *__restrict__ partials,
    int32_t *__restrict__ tickets, float alpha, float beta) {
    constexpr int BAND = 1 << BAND_LOG2;
    constexpr int BROWS = 1 << ROWS_LOG2;
    constexpr XbBits kBits = xb_bits(BAND_LOG2, ROWS_LOG2);
    constexpr uint32_t kColMask = (1u << kBits.col) - 1u;
    constexpr uint32_t kRankMask = (1u << kBits.rank) - 1u;
    constexpr uint32_t kDummyRank = kBits.dummy_rank();
    constexpr uint32_t kDummyWord = kBits.dummy_word();
    constexpr int kWaves = THREADS / 64;
    constexpr int kER = EA < 4 ? 4 : 8;   // entry ring = loop unroll
    constexpr int kXR = GA < 4 ? 4 : 8;   // x-value ring
    static_assert(GA >= 1 && GA < EA && EA < kER && kER % kXR == 0, "lookaheads");
    static_assert(BROWS % (4 * THREADS) == 0, "accumulator init in float4 per thread");
    __shared__ __attribute__((aligned(16))) float yacc[BROWS + 64];   // + a scratch slot per lane
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int32_t b = blockIdx.x / n_slabs;
    const int32_t slab = blockIdx.x - b * n_slabs;
    const int32_t p_first = slab * slab_bands;
    const int32_t nb = min(slab_bands, n_bands - p_first);
    if (!(ABL & 4)) handoff_started(tickets + (int64_t)b * kCtlWords, n_slabs);
    const int32_t r0 = b * block_rows;
    const int32_t nr = min(block_rows, n_rows - r0);
    const int32_t *csg = chunk_start + (int64_t)b * n_bands + p_first;
    const int32_t c_first = csg[0];
    const int32_t c_last = csg[nb];
    const int64_t x0 = (int64_t)p_first * BAND;
    const __amdgpu_buffer_rsrc_t xr_src = rsrc(x + x0, (uint64_t)(n_cols - x0) * 4);
    const __amdgpu_buffer_rsrc_t w_src =
        rsrc(word + (int64_t)c_first * 64, (uint64_t)(c_last - c_first) * 256);
    const __amdgpu_buffer_rsrc_t v_src =
        rsrc(val + (int64_t)c_first * 64, (uint64_t)(c_last - c_first) * 256);
    // Chunk table window in registers (as above).
    int32_t cw = 0;
    int32_t cs_lo = csg[min(lane, nb)];
    int32_t cs_hi = csg[min(64 + lane, nb)];
    auto advance_cs_window = [&]() {
        cw += 64;
        cs_lo = cs_hi;
        cs_hi = csg[min(cw + 64 + lane, nb)];
    };
    auto cs_at = [&](int32_t i) -> int32_t {
        const int32_t j = i - cw;
        const int32_t lo = __builtin_amdgcn_readlane(cs_lo, j & 63);
        const int32_t hi = __builtin_amdgcn_readlane(cs_hi, j & 63);
        return (j < 64 ? lo : hi) - c_first;
    };
    // Chunk c0+wave+16k of band p; slots past the band read 0 = a dummy (see above).
    auto load_entries = [&](int32_t p, uint32_t *w, float *v) {
        const bool inb = p < nb;
        const int32_t c0 = inb ? cs_at(p) : 0;
        const int32_t c1 = inb ? cs_at(p + 1) : 0;
#pragma unroll
        for (int k = 0; k < CAP; ++k) {
            const int32_t c = c0 + wave + k * kWaves;
            const uint32_t off = c < c1 ? 4u * (uint32_t)(c * 64 + lane) : 0xFFFFFF00u;
            w[k] = __builtin_amdgcn_raw_buffer_load_b32(w_src, off, 0, kAuxNt);
            v[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(v_src, off, 0, kAuxNt));
        }
    };
    // x values of band p's entries (dummies decode to column 0 of the band: a
    // harmless in-range read; bands past the tile read nothing).
    auto gather_x = [&](int32_t p, const uint32_t *w, float *xg) {
        const uint32_t pb = p < nb ? (uint32_t)p * BAND : 0u;
#pragma unroll
        for (int k = 0; k < CAP; ++k) {
            const uint32_t col = (w[k] ^ kDummyWord) & kColMask;
            const uint32_t off = p < nb ? 4u * (pb + col) : 0xFFFFFF00u;
            if (ABL & 1)
                xg[k] = __uint_as_float(off);
            else
                xg[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr_src, off, 0, 0));
        }
    };
    auto shr1 = [](float v) {
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, false));
    };
    auto shl1 = [](uint32_t v) {
        return (uint32_t)__builtin_amdgcn_update_dpp((int)kDummyRank, (int)v, 0x130, 0xF, 0xF, false);
    };
    auto apply_band = [&](const float *xv, const uint32_t *wa, const float *va) {
        float yv[CAP];
        uint32_t rk[CAP], rl[CAP];
        bool live[CAP];
        bool more = false;
#pragma unroll
        for (int k = 0; k < CAP; ++k) {
            const uint32_t wd = wa[k] ^ kDummyWord;
            rk[k] = (wd >> kBits.col) & kRankMask;
            live[k] = rk[k] != kDummyRank;
            rl[k] = wd >> (kBits.col + kBits.rank);
            yv[k] = yacc[rl[k]];
            more |= live[k] && rk[k] > 0;
        }
        pin_one<CAP>(yv);
        float t[CAP], acc[CAP];
#pragma unroll
        for (int k = 0; k < CAP; ++k) {
            t[k] = __fmul_rn(xv[k], __fmul_rn(va[k], alpha));
            acc[k] = __fadd_rn(yv[k], t[k]);
        }
        if (__any(more)) {
            for (uint32_t r = 1;; ++r) {
                bool again = false;
#pragma unroll
                for (int k = 0; k < CAP; ++k) {
                    const float prev = shr1(acc[k]);
                    if (rk[k] == r) acc[k] = __fadd_rn(prev, t[k]);
                    again |= live[k] && rk[k] > r;
                }
                if (!__any(again)) break;
            }
        }
#pragma unroll
        for (int k = 0; k < CAP; ++k) {
            const bool last = live[k] && shl1(rk[k]) != rk[k] + 1u;
            yacc[last ? rl[k] : (uint32_t)(BROWS + lane)] = acc[k];
        }
    };

    // Accumulators: beta*y (slab 0) or -0.0 (see above), all loads in flight at once.
    constexpr int kQ = BROWS / (4 * THREADS);
    const bool y_vec = ((uintptr_t)(y + r0) & 15) == 0;
    if (slab == 0) {
        const __amdgpu_buffer_rsrc_t yi_src = rsrc(y + r0, (uint64_t)nr * 4);
        float4 v[kQ];
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const uint32_t o = 16u * (uint32_t)(tid + q * THREADS);
            if (y_vec) {
                const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(yi_src, o, 0, 0);
                v[q] = make_float4(__uint_as_float(u.x), __uint_as_float(u.y),
                                   __uint_as_float(u.z), __uint_as_float(u.w));
            } else {
                v[q] = make_float4(
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o, 0, 0)),
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 4, 0, 0)),
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 8, 0, 0)),
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 12, 0, 0)));
            }
        }
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            if (beta != 1.0f)
                v[q] = make_float4(__fmul_rn(v[q].x, beta), __fmul_rn(v[q].y, beta),
                                   __fmul_rn(v[q].z, beta), __fmul_rn(v[q].w, beta));
            *reinterpret_cast<float4 *>(&yacc[4 * (tid + q * THREADS)]) = v[q];
        }
    } else {
#pragma unroll
        for (int q = 0; q < kQ; ++q)
            *reinterpret_cast<float4 *>(&yacc[4 * (tid + q * THREADS)]) = make_float4(-0.f, -0.f, -0.f, -0.f);
    }

    // Rings with static roles: entries of band q in W/V[q % kER], its x values in
    // XG[q % kER].  Prologue: the loads the loop expects in flight, in its order
    // (band q issues entries q+EA, then gathers q+GA).
    uint32_t W[kER][CAP];
    float V[kER][CAP];
    float XG[kXR][CAP];
#pragma unroll
    for (int q = -EA; q < 0; ++q) {
        load_entries(q + EA, W[(q + EA) % kER], V[(q + EA) % kER]);
        if (q + GA >= 0) gather_x(q + GA, W[(q + GA + kER) % kER], XG[(q + GA + kER) % kXR]);
    }
    __syncthreads();
    const int32_t nbu = (nb + kER - 1) / kER * kER;   // whole groups (no early exit)
    for (int32_t p = 0; p < nbu; p += kER) {
#pragma unroll
        for (int u = 0; u < kER; ++u) {
            if (p + u + EA >= cw + 64) advance_cs_window();
            load_entries(p + u + EA, W[(u + EA) % kER], V[(u + EA) % kER]);
            gather_x(p + u + GA, W[(u + GA) % kER], XG[(u + GA) % kXR]);
            if (ABL & 2) {
#pragma unroll
                for (int k = 0; k < CAP; ++k) asm volatile("" ::"v"(W[u][k]), "v"(V[u][k]), "v"(XG[u % kXR][k]));
            } else {
                apply_band(XG[u % kXR], W[u], V[u]);
            }
            __syncthreads();
        }
    }

    if (n_slabs == 1 || (ABL & 4)) {
        const int32_t nv = y_vec ? (nr & ~3) : 0;
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int32_t i = 4 * (tid + q * THREADS);
            if (i < nv) *reinterpret_cast<float4 *>(y + r0 + i) = *reinterpret_cast<const float4 *>(&yacc[i]);
        }
        for (int32_t i = nv + tid; i < nr; i += THREADS) y[r0 + i] = yacc[i];
        return;
    }
    __shared__ int32_t s_word[3];
    slab_handoff<THREADS>(yacc, tickets + (int64_t)b * kCtlWords, s_word, y, partials, n_rows, r0,
                          nr, slab, n_slabs, y_vec);
}

// SM_XBAND_GLOOK = "EA,GA" picks the lookaheads (development A/B; default 5,2).
template <int THREADS, int BAND_LOG2, int ROWS_LOG2, int CAP>
hipError_t launch_gtiles(const XbandDev &xb, int32_t n_rows, int32_t n_cols, const float *x,
                         float *y, float alpha, float beta, hipStream_t s) {
#define SM_GBL(EA, GA)                                                                            \
    hipLaunchKernelGGL((spmv_gband_kernel<THREADS, BAND_LOG2, ROWS_LOG2, CAP, EA, GA>),           \
                       dim3((unsigned)((int64_t)xb.n_blocks * xb.n_slabs)), dim3(THREADS), 0, s,  \
                       n_rows, n_cols, xb.block_rows, xb.n_bands, xb.n_slabs, xb.slab_bands,     \
                       xb.d_chunk_start, xb.d_word, xb.d_val, x, y, xb.d_partials, xb.d_tickets, \
                       alpha, beta)
#ifdef SM_DEV
    static const int look = [] {
        const char *e = dev_env("SM_XBAND_GLOOK");
        if (!e) return 52;
        const int ea = atoi(e), ga = strchr(e, ',') ? atoi(strchr(e, ',') + 1) : 0;
        return 10 * ea + ga;
    }();
    static const int abl = [] {
        const char *e = dev_env("SM_GBAND_ABLATE");
        return e ? atoi(e) : 0;
    }();
    if (abl) {
        switch (abl) {
#define SM_GBA(A)                                                                                  \
    case A:                                                                                        \
        hipLaunchKernelGGL((spmv_gband_kernel<THREADS, BAND_LOG2, ROWS_LOG2, CAP, 5, 2, A>),       \
                           dim3((unsigned)((int64_t)xb.n_blocks * xb.n_slabs)), dim3(THREADS), 0, s, \
                           n_rows, n_cols, xb.block_rows, xb.n_bands, xb.n_slabs, xb.slab_bands, \
                           xb.d_chunk_start, xb.d_word, xb.d_val, x, y, xb.d_partials, xb.d_tickets, \
                           alpha, beta);                                                           \
        return hipGetLastError();
        SM_GBA(1) SM_GBA(2) SM_GBA(3) SM_GBA(4) SM_GBA(7)
#undef SM_GBA
        default: return hipErrorInvalidValue;
        }
    }
    switch (look) {
    case 32: SM_GBL(3, 2); break;
    case 62: SM_GBL(6, 2); break;
    case 63: SM_GBL(6, 3); break;
    case 73: SM_GBL(7, 3); break;
    default: SM_GBL(5, 2); break;
    }
#else
    SM_GBL(5, 2);   // entries 5 bands ahead, x gathers 2
#endif
#undef SM_GBL
    return hipGetLastError();
}

template <int THREADS, int BAND_LOG2, int ROWS_LOG2>
hipError_t launch_gkind(const XbandDev &xb, int32_t n_rows, int32_t n_cols, const float *x,
                        float *y, float alpha, float beta, hipStream_t s) {
    const int64_t cap = (xb.max_chunks_per_band + THREADS / 64 - 1) / (THREADS / 64);
#define SM_GBT(C) launch_gtiles<THREADS, BAND_LOG2, ROWS_LOG2, C>(xb, n_rows, n_cols, x, y, alpha, beta, s)
    if (cap <= 1) return SM_GBT(1);
    if (cap <= 2) return SM_GBT(2);
    if (cap <= 3) return SM_GBT(3);
    if (cap <= 4) return SM_GBT(4);
    if (cap <= kXbMaxCap) return SM_GBT(5);
#undef SM_GBT
    return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_spmv_xband(const XbandDev &xb, int32_t n_rows, int32_t n_cols, const float *x,
                             float *y, float alpha, float beta, hipStream_t s) {
    if (xb.n_blocks <= 0) return hipSuccess;
    if (xb.n_bands > kXbMaxBands || xb.n_slabs < 1 || xb.slab_bands < 1 ||
        (int64_t)xb.n_slabs * xb.slab_bands < xb.n_bands ||
        (int64_t)(xb.n_slabs - 1) * xb.slab_bands >= xb.n_bands ||
        (xb.n_slabs > 1 && (!xb.d_partials || !xb.d_tickets)))
        return hipErrorInvalidValue;
    hipError_t e = hipErrorInvalidValue;
    if (xb.kind == kXbExact && xb.band_cols == 1 << kXbExactBandLog2 &&
        xb.block_rows <= 1 << kXbExactRowsLog2)
        e = launch_kind<kXbThreads, kXbExactBandLog2, kXbExactRowsLog2>(xb, n_rows, n_cols, x, y, alpha, beta, s);
    else if (xb.kind == kXbBlocked && xb.band_cols == 1 << kXbBlockedBandLog2 &&
             xb.block_rows <= 1 << kXbBlockedRowsLog2)
        e = launch_kind<kXbThreads, kXbBlockedBandLog2, kXbBlockedRowsLog2>(xb, n_rows, n_cols, x, y, alpha, beta, s);
    else if (xb.kind == kXbGather && xb.band_cols == 1 << kXbGatherBandLog2 &&
             xb.block_rows <= 1 << kXbGatherRowsLog2)
        e = launch_gkind<kXbThreads, kXbGatherBandLog2, kXbGatherRowsLog2>(xb, n_rows, n_cols, x, y, alpha, beta, s);
    else if (xb.kind == kXbGather && xb.band_cols == 1 << (kXbGatherWideBandLog2 - 1) &&
             xb.block_rows <= 1 << kXbGatherRowsLog2)
        e = launch_gkind<kXbThreads, kXbGatherWideBandLog2 - 1, kXbGatherRowsLog2>(xb, n_rows, n_cols, x, y, alpha, beta, s);
    else if (xb.kind == kXbGather && xb.band_cols == 1 << kXbGatherWideBandLog2 &&
             xb.block_rows <= 1 << kXbGatherRowsLog2)
        e = launch_gkind<kXbThreads, kXbGatherWideBandLog2, kXbGatherRowsLog2>(xb, n_rows, n_cols, x, y, alpha, beta, s);
    return e;
}

}  // namespace smamd
