// kernels_band2.hip -- SpMV over the balanced-band layout (band2.cpp, xband.h).
//
// One workgroup (1024 threads, 16 waves) per tile = (block of <= 16384 rows, slab of
// columns), one per CU.  A tile's bands are column windows holding a fixed number of
// 64-entry chunks (dummies pad the last); the block's row sums live in LDS.  Entries:
// band2 8 bytes per term (word + fp32 value), cband 4 bytes (a codebook word, the value
// looked up in an LDS copy of the <= 255-entry table scaled by alpha).  Two geometries:
//
//   dma3 (kB2Dma3Cb / kB2Dma3B2, the default): wave 15 is a loader -- it stages the x
//     windows (7680 columns) by LDS-DMA into three buffers, two bands ahead, and applies
//     nothing; waves 0..14 apply chunks 2w, 2w+1 of 30-chunk bands and never hold x in
//     registers.  Per band: apply, load the entries of band q+2, barrier.
//   wide (kB2Wide, the fallback when dma3's bands would be < 70 % full): every wave
//     applies chunks 2w, 2w+1 of 32-chunk bands of 8192 columns and stages x itself
//     through registers (two float4 per lane): load window q+2, issue band q's LDS reads,
//     store window q+1 into the free buffer (after the reads, so they do not queue behind
//     16 waves' stores), finish band q, load the entries of band q+2, barrier.
//
// A chunk's terms are added to the LDS sums in rank rounds (a row's segment runs up
// consecutive lanes by DPP, its last lane writes; no two lanes touch one row in a round, no
// atomics).  Summation order: bands ascend in column, a row's terms inside a band ascend in
// column, so inside a tile every row is summed in the reference's order (kernel.cc:780-796,
// per output ascending column, kernel.cc:791 for the term).  One slab: the tile starts from
// beta*y -- bit-identical to the reference.  Several: every slab tile starts from -0.0 and the
// slab hand-off (xband_dev.h slab_handoff_epoch, beta-last) forms beta*y and adds the slab
// sums in slab order -- within the Sum|terms| bound, deterministic.
//
// The variants measured slower over rounds 2-5 (tall, wide3, half2 and dma3-tall
// geometries, several loader waves, x by LDS-DMA in the wide geometry, early entry loads,
// x / codebook prefetch, the row-owner bands) are gone from this file; DESIGN.md §3.4b
// keeps their numbers and the commits that held them.
#include "sm_internal.h"
#include "xband.h"
#include "xband_dev.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

namespace smamd {
namespace {

constexpr int kB2Threads = 1024;
#ifdef SM_DEV
// PROF 1 (development builds, SM_BAND2_PROF=1, dma3): lane 0 of every wave adds the cycles
// (s_memtime) of each phase of the band loop -- applying waves: [0] entry wait, [1] apply,
// [2] barrier; the loader: [3] DMA issue, [4] its wait, [5] barrier; [6] bands, [7] waves.
__device__ unsigned long long g_b2_prof[8];
// PROF 2 (SM_BAND2_PROF=2): wall clock (s_memrealtime, 100 MHz) of every tile's start, loop
// end and finish, from thread 0.
// PROF 2 also stamps the hand-off (xband_dev.h slab_handoff_epoch): [3] published and drained,
// [4] arrival add returned, [5] every sibling seen, [6] combine stores drained.
constexpr int kTs = 8;
__device__ unsigned long long g_b2_ts[kTs * 4096];
#endif
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Lookaheads (bands): x windows (wide) and entries.  Two bands of cover suffice; 3-8
// measured slower.
constexpr int kXAhead = 2;
constexpr int kEAhead = 2;
constexpr int kApplyPrio = 2;    // s_setprio of the applying waves' LDS work
constexpr int kLoaderPrio = 3;   // the dma3 loader outranks them (its DMA issue goes first)
// Wide cband: the table in 32 copies, lane l reads copy l % 32, so the reads of a 32-lane
// group spread over the banks whatever the ids (37.3 vs 38.1 us with 16, 39.1 with 8).
constexpr int kWideTabCopies = 32;

// CB: the cband encoding (xband.h): one 32-bit word per term, values from the codebook
// `table` (<= 255 entries), scaled by alpha once into LDS.  GEO: 0 wide, 4 dma3.
template <bool CB, int GEO, int PROF>
__global__ __launch_bounds__(kB2Threads) void spmv_band2_kernel(
    int32_t n_rows, int32_t n_cols, int32_t block_rows, int32_t n_slabs,
    const int32_t *__restrict__ tile_band_start, const int32_t *__restrict__ band_clo,
    const uint32_t *__restrict__ ent, const float *__restrict__ table, int32_t table_size,
    const float *__restrict__ x, float *__restrict__ y, float *__restrict__ partials,
    int32_t *__restrict__ ctl, float alpha, float beta) {
    static_assert(GEO == 0 || GEO == 4, "wide or dma3");
    constexpr bool kLd = GEO == 4;   // dma3: wave kLdWave stages x, the others apply
    constexpr B2Geom G = kLd ? (CB ? kB2Dma3Cb : kB2Dma3B2) : kB2Wide;
    constexpr int kLdWave = kB2Threads / 64 - 1;
    constexpr int CPW = 2;   // chunks per applying wave per band
    static_assert(G.chunks() == CPW * (kLd ? kLdWave : kB2Threads / 64), "every applying wave holds two chunks");
    constexpr int BROWS = G.block_rows;
    constexpr int W = G.window;
    constexpr int XV = (W + 4 * kB2Threads - 1) / (4 * kB2Threads);   // float4 of x per lane (wide)
    constexpr int kB2Col = G.col_bits;                                // band2 word fields
    constexpr uint32_t kB2Dummy = G.dummy_word();
    constexpr uint32_t kColMask = (1u << kB2Col) - 1u;
    constexpr uint32_t kRankMask = (1u << kB2RankBits) - 1u;
    // Wide band2 keeps a scratch slot per lane for its dummy lanes' writes; the other forms
    // write only live lanes and use the LDS nearly to the last byte.
    constexpr bool kScratch = !CB && GEO == 0;
    // Rings with static roles: x window p+AX and the entries of band p+AE are loaded at band p
    // into the slots band p just freed.  Loop unroll U: both rings and (dma3) the three x
    // buffers divide it, so no ring index is dynamic (a branch around a ring register makes
    // hipcc copy registers and drain vmcnt).
    constexpr int AX = kXAhead, AE = kEAhead;
    constexpr int kXBuf = kLd ? 3 : 2;
    constexpr int U = kLd ? 6 : 2;
    static_assert(U % AX == 0 && U % AE == 0 && U % kXBuf == 0, "ring sizes divide the unroll");
    static_assert(W % 4 == 0 && XV * 4 * kB2Threads >= W, "float4 slots cover the window");
    static_assert(!kLd || W % 256 == 0, "dma3 windows are whole 1 KiB pieces");
    __shared__ __attribute__((aligned(16))) float xs[kXBuf][W];
    __shared__ __attribute__((aligned(16))) float yacc[BROWS + (kScratch ? 64 : 0)];
    // cband: fl(table[id] * alpha) (0 past the table) in kTabCopies copies, entry id of copy c
    // at kTabCopies * id + c; lane l reads copy l % kTabCopies (dma3: 4 copies, the builder
    // places each term's lane against the table banks too).
    constexpr int kTabCopies = GEO == 0 ? kWideTabCopies : G.tab_copies;
    __shared__ float tab[CB ? 256 * kTabCopies : 1];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int32_t wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR)
#ifdef SM_DEV
    if constexpr (PROF == 2) {
        if (threadIdx.x == 0 && blockIdx.x < 4096) g_b2_ts[kTs * blockIdx.x] = wall_clock64();
    }
#endif
    [[maybe_unused]] unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    [[maybe_unused]] unsigned long long tk = PROF == 1 ? clock64() : 0;
    auto mark_phase = [&](int k) {
        if constexpr (PROF == 1) {
            const unsigned long long now = clock64();
            ph[k] += now - tk;
            tk = now;
        }
    };
    const int32_t t = blockIdx.x;
    const int32_t b = t / n_slabs;
    const int32_t slab = t - b * n_slabs;
    const uint64_t old_started = handoff_begin(ctl + (int64_t)b * kCtlWords, n_slabs);
    const int32_t g0 = tile_band_start[t];
    const int32_t nb = tile_band_start[t + 1] - g0;
    const int32_t r0 = b * block_rows;
    const int32_t nr = min(block_rows, n_rows - r0);
    const __amdgpu_buffer_rsrc_t x_src = rsrc(x, (uint64_t)n_cols * 4);
    constexpr uint32_t kBandBytes = (CB ? 4u : 8u) * 64u * (uint32_t)G.chunks();   // entries of one band
    // Threads that hold entries (dma3: all but the loader wave, whose loads go past the range).
    constexpr int kApplyThreads = 64 * G.chunks() / CPW;
    static_assert(kApplyThreads <= kB2Threads && kBandBytes % kApplyThreads == 0, "whole entry slots per lane");
    const __amdgpu_buffer_rsrc_t e_src = rsrc(ent + (int64_t)g0 * (kBandBytes / 4), (uint64_t)nb * kBandBytes);
    // Band windows: lane l holds clo of bands cw + l (lo) and cw + 64 + l (hi), read by
    // readlane; the window advances by 64 bands when the x loads reach its hi half.
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

    // Wide: x window q into registers, float4 slots tid (+ 1024) of [clo_q, clo_q + W);
    // windows past the tile and slots past W read nothing (offset past the descriptor).
    auto load_x = [&](int32_t q, float4 *xr) {
        const int32_t c = q < nb ? clo_at(q) : 0;
#pragma unroll
        for (int k = 0; k < XV; ++k) {
            const int32_t slot = 4 * (tid + k * kB2Threads);
            const uint32_t off = q < nb && slot < W ? 4u * (uint32_t)(c + slot) : 0xFFFFFFF0u;
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(x_src, off, 0, 0);
            xr[k] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                                __uint_as_float(v.w));
        }
    };
    auto store_x = [&](int buf, const float4 *xr) {
#pragma unroll
        for (int k = 0; k < XV; ++k) {
            const int32_t slot = 4 * (tid + k * kB2Threads);
            if (W % (4 * kB2Threads) == 0 || slot < W) *reinterpret_cast<float4 *>(&xs[buf][slot]) = xr[k];
        }
    };
    // dma3: the loader wave's LDS-DMA of the window starting at column c into buffer buf,
    // W / 256 pieces of 1 KiB (one wave-instruction each).
    const uint32_t xs_lds = (uint32_t)(size_t)(__attribute__((address_space(3))) float *)&xs[0][0];
    auto dma_win = [&](int32_t c, int32_t buf) {
#pragma unroll
        for (int m = 0; m < W / 256; ++m) {
            const uint32_t voff = 4u * (uint32_t)(c + m * 256 + lane * 4);
            const uint32_t lds = __builtin_amdgcn_readfirstlane(xs_lds + 4u * (uint32_t)(buf * W + m * 256));
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(voff), "s"(x_src), "s"(lds)
                : "memory");
        }
    };
    // Entries of band q: band2 {word 2w, word 2w+1, value 2w, value 2w+1}, cband {word 2w,
    // word 2w+1} for this lane; past the tile (and the dma3 loader): zeros = dummies.
    using EV = typename std::conditional<CB, u32x2, u32x4>::type;
    auto load_e = [&](int32_t q) -> EV {
        const uint32_t off = (kApplyThreads < kB2Threads && tid >= kApplyThreads)
                                 ? 0xFFFFFFF0u
                                 : kBandBytes * (uint32_t)q + (kBandBytes / kApplyThreads) * (uint32_t)tid;
        if constexpr (CB)
            return __builtin_amdgcn_raw_buffer_load_b64(e_src, off, 0, kAuxNt);
        else
            return __builtin_amdgcn_raw_buffer_load_b128(e_src, off, 0, kAuxNt);
    };

    auto shr1 = [](float v) {   // lane i <- lane i-1 (lane 0 never has rank >= 1)
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, false));
    };
    auto shl1 = [](uint32_t v) {   // lane i <- lane i+1; lane 63 <- the dummy rank
        return (uint32_t)__builtin_amdgcn_update_dpp((int)kB2DummyRank, (int)v, 0x130, 0xF, 0xF, false);
    };
    // band2 apply in two steps (b2_read issues the four LDS reads, b2_finish adds and writes;
    // the wide loop stores the next x window between them).
    struct B2State {
        float xv[2], yv[2], va[2];
        uint32_t rk[2], rl[2];
        bool live[2];
        bool more;
    };
    auto b2_read = [&](const float *xb, u32x4 e) -> B2State {
        __builtin_amdgcn_s_setprio(kApplyPrio);
        const uint32_t wd[2] = {e.x ^ kB2Dummy, e.y ^ kB2Dummy};
        B2State st;
        st.va[0] = __uint_as_float(e.z);
        st.va[1] = __uint_as_float(e.w);
        st.more = false;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            st.rk[k] = (wd[k] >> kB2Col) & kRankMask;
            st.live[k] = st.rk[k] != kB2DummyRank;
            st.rl[k] = wd[k] >> (kB2Col + kB2RankBits);   // dummies decode to row 0, column 0
            st.xv[k] = xb[wd[k] & kColMask];
            st.yv[k] = yacc[st.rl[k]];
            st.more |= st.live[k] && st.rk[k] > 0;
        }
        return st;
    };
    auto b2_finish = [&](B2State st) {
        float *xv = st.xv, *yv = st.yv;
        const uint32_t *rk = st.rk, *rl = st.rl;
        const bool *live = st.live;
        // Materialise all four reads before any write (one LDS wait per band).
        asm volatile("" : "+v"(xv[0]), "+v"(xv[1]), "+v"(yv[0]), "+v"(yv[1]));
        float tm[2], acc[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            tm[k] = __fmul_rn(xv[k], __fmul_rn(st.va[k], alpha));
            acc[k] = __fadd_rn(yv[k], tm[k]);
        }
        if (__any(st.more)) {
            for (uint32_t r = 1;; ++r) {
                bool again = false;
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const float prev = shr1(acc[k]);
                    if (rk[k] == r) acc[k] = __fadd_rn(prev, tm[k]);
                    again |= live[k] && rk[k] > r;
                }
                if (!__any(again)) break;
            }
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {   // the segment's last lane writes its row
            const bool last = live[k] && shl1(rk[k]) != rk[k] + 1u;
            if constexpr (kScratch)
                yacc[last ? rl[k] : (uint32_t)(BROWS + lane)] = acc[k];   // every lane writes
            else if (last)
                yacc[rl[k]] = acc[k];
        }
        __builtin_amdgcn_s_setprio(0);
    };

    // Lane select by an SGPR lane mask (v_cndmask_b32 with the mask as its condition):
    // lane i takes b where bit i of m is set, else a.
    auto sel = [](uint64_t m, float a, float bb) -> float {
        float r;
        asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(bb), "s"(m));
        return r;
    };
    // cband: row = chunk base (lane 0's header) + offset.  A segment's running sum moves up
    // one lane per round in lane (= column) order; the lanes a round updates are an SGPR
    // mask: the continuations whose predecessor finished last round.
    constexpr uint32_t kCbCol = (1u << G.cb_col) - 1u;
    constexpr uint32_t kCbDummy = G.cb_dummy_word();
    constexpr int kCbOffSh = G.cb_off_shift();
    constexpr uint32_t kCbOffM = G.cb_off_mask();
    struct CbState {
        float xv[CPW], yv[CPW], tv[CPW];
        uint32_t rl[CPW];
        uint64_t live[CPW], cont[CPW];
    };
    auto cb_read = [&](const float *xb, EV e) -> CbState {
        __builtin_amdgcn_s_setprio(kApplyPrio);
        CbState st;
#pragma unroll
        for (int k = 0; k < CPW; ++k) {
            const uint32_t wd = e[k] ^ kCbDummy;
            const uint32_t h = (uint32_t)__builtin_amdgcn_readlane((int)wd, 0);
            const uint32_t base = (h & kCbCol) | (((h >> kCbOffSh) & kCbOffM) << G.cb_col);
            const uint32_t id = (wd >> G.cb_col) & kCbDummyId;
            st.live[k] = __ballot(id != kCbDummyId);
            st.cont[k] = __ballot((int32_t)wd < 0);
            st.rl[k] = base + ((wd >> kCbOffSh) & kCbOffM);
            st.xv[k] = xb[wd & kCbCol];
            st.tv[k] = tab[id * kTabCopies + (lane & (kTabCopies - 1))];
            st.yv[k] = yacc[st.rl[k]];
        }
        return st;
    };
    auto cb_finish = [&](CbState st) {
        float *xv = st.xv, *yv = st.yv, *tv = st.tv;
        // Materialise all reads before any write (one LDS wait per band).
        asm volatile("" : "+v"(xv[0]), "+v"(xv[1]), "+v"(yv[0]), "+v"(yv[1]), "+v"(tv[0]), "+v"(tv[1]));
        float tm[CPW], acc[CPW];
        uint64_t R[CPW];
#pragma unroll
        for (int k = 0; k < CPW; ++k) {
            tm[k] = __fmul_rn(xv[k], tv[k]);
            acc[k] = __fadd_rn(yv[k], tm[k]);
            R[k] = st.cont[k] & ~(st.cont[k] << 1);
        }
        while ((R[0] | R[1]) != 0) {
#pragma unroll
            for (int k = 0; k < CPW; ++k) {
                acc[k] = sel(R[k], acc[k], __fadd_rn(shr1(acc[k]), tm[k]));
                R[k] = st.cont[k] & (R[k] << 1);
            }
        }
#pragma unroll
        for (int k = 0; k < CPW; ++k) {   // the segment's last lane writes its row
            const uint64_t last = st.live[k] & ~(st.cont[k] >> 1);
            if ((last >> lane) & 1) yacc[st.rl[k]] = acc[k];
        }
        __builtin_amdgcn_s_setprio(0);
    };
    using RState = typename std::conditional<CB, CbState, B2State>::type;
    auto read = [&](const float *xb, EV e) -> RState {
        if constexpr (CB) return cb_read(xb, e);
        else return b2_read(xb, e);
    };
    auto finish = [&](RState st) {
        if constexpr (CB) cb_finish(st);
        else b2_finish(st);
    };

    // Prologue, ordered so its memory latencies overlap: the first windows' x and entry loads
    // go out first, then the codebook and (slab 0) y loads; the LDS writes of all of them
    // follow, so the tile waits about one memory latency before its first band instead of one
    // per kind of load (vmcnt retires in issue order).  Rings: x window q in X[q % AX],
    // entries of band q in E[q % AE]; the wide prologue = virtual bands -U..-1 (their loads in
    // the loop's order), so the loads pending at the loop header are in the order the loop's
    // back edge leaves them.
    [[maybe_unused]] float4 X[AX][XV];
    EV E[AE];
    if constexpr (kLd) {
#pragma unroll
        for (int v = 0; v < AE; ++v) E[v] = load_e(v);
        if (wid == kLdWave) {   // windows 0 and 1; waited for (with everything) below
            if (nb > 0) dma_win(clg[0], 0);
            if (nb > 1) dma_win(clg[1], 1);
        }
    } else {
#pragma unroll
        for (int v = -U; v < 0; ++v) {
            if (v + AX >= 0) load_x(v + AX, X[v + AX]);
            if (v + AE >= 0) E[v + AE] = load_e(v + AE);
        }
    }
    // Codebook: fl(table[id] * alpha), loaded now, written below.
    constexpr bool kTabSmall = 256 * kTabCopies < 4 * kB2Threads;   // at most two entries per thread
    constexpr int kPer = kTabSmall ? 1 : 256 * kTabCopies / kB2Threads;   // copies written per thread
    float tab_v = 0.0f;
    if constexpr (CB && !kTabSmall) {
        static_assert(kPer % 4 == 0 && kTabCopies % kPer == 0, "whole float4 of one entry");
        const int id = tid / (kTabCopies / kPer);   // one entry per thread
        tab_v = id < table_size ? table[id] : 0.0f;
    }
    // Accumulators: beta*y (slab 0 of a one-slab layout, or of any layout without SM_B2_BL) or
    // -0.0 (the identity of fp32 addition: a row without terms in this slab keeps the sign of a
    // zero y), all loads in flight.
    constexpr int kQ = BROWS / (4 * kB2Threads);
    const bool y_vec = ((uintptr_t)(y + r0) & 15) == 0;
    const bool y_first = slab == 0 && (n_slabs == 1 || !SM_B2_BL);
    float4 yv[kQ];
    if (y_first) {
        const __amdgpu_buffer_rsrc_t yi_src = rsrc(y + r0, (uint64_t)nr * 4);
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const uint32_t o = 16u * (uint32_t)(tid + q * kB2Threads);
            if (y_vec) {
                const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(yi_src, o, 0, 0);
                yv[q] = make_float4(__uint_as_float(u.x), __uint_as_float(u.y),
                                    __uint_as_float(u.z), __uint_as_float(u.w));
            } else {
                yv[q] = make_float4(
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o, 0, 0)),
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 4, 0, 0)),
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 8, 0, 0)),
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yi_src, o + 12, 0, 0)));
            }
        }
    }
    if constexpr (CB) {
        if constexpr (kTabSmall) {
            for (int i = tid; i < 256 * kTabCopies; i += kB2Threads) {
                const int id = i / kTabCopies;
                tab[i] = id < table_size ? __fmul_rn(table[id], alpha) : 0.0f;
            }
        } else {
            const int id = tid / (kTabCopies / kPer);
            const float v = id < table_size ? __fmul_rn(tab_v, alpha) : 0.0f;
#pragma unroll
            for (int j = 0; j < kPer; j += 4)
                *reinterpret_cast<float4 *>(&tab[kPer * tid + j]) = make_float4(v, v, v, v);
        }
    }
    if (y_first) {
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            if (beta != 1.0f)
                yv[q] = make_float4(__fmul_rn(yv[q].x, beta), __fmul_rn(yv[q].y, beta),
                                    __fmul_rn(yv[q].z, beta), __fmul_rn(yv[q].w, beta));
            *reinterpret_cast<float4 *>(&yacc[4 * (tid + q * kB2Threads)]) = yv[q];
        }
    } else {
#pragma unroll
        for (int q = 0; q < kQ; ++q)
            *reinterpret_cast<float4 *>(&yacc[4 * (tid + q * kB2Threads)]) = make_float4(-0.f, -0.f, -0.f, -0.f);
    }
    if constexpr (kLd) {
        if (wid == kLdWave) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        store_x(0, X[0]);
    }
    __syncthreads();
    // The commit check's snapshot (xband_dev.h slab_handoff_epoch): read now, used after the
    // band loop, so its round trip hides behind the loop.
    const uint64_t snap = handoff_snapshot(ctl + (int64_t)b * kCtlWords, n_slabs);

    // Whole groups of U bands.  Steps past the tile's last band see only dummy entries (their
    // loads go past the descriptors: no memory request) and skip the barrier -- a uniform
    // branch; the dummies write nothing but the x buffers nobody reads any more (band2: and
    // the scratch slots).
    const int32_t nbu = (nb + U - 1) / U * U;
    mark_phase(0);
    if constexpr (PROF == 1) ph[0] = 0;   // the prologue is not a band phase
    if constexpr (kLd) {
        if (wid == kLdWave) {
            // Band q: DMA window q+2 into the buffer window q-1 left (every wave passed band
            // q-1's barrier), then wait until window q+1 has landed -- the 30 pieces just issued
            // may stay in flight -- and meet the others at the barrier.  The windows' first
            // columns come by scalar loads one band ahead (a vector load here would make hipcc
            // wait for the whole DMA queue before reading it).
            int32_t c_next = nb > 2 ? clg[2] : 0;
            __builtin_amdgcn_s_setprio(kLoaderPrio);
            for (int32_t q = 0; q < nb; ++q) {
                if (q + 2 < nb) {
                    const int32_t c = c_next;
                    const int32_t qn = __builtin_amdgcn_readfirstlane(q + 3);
                    if (qn < nb) c_next = clg[qn];
                    mark_phase(5);
                    dma_win(c, (q + 2) % 3);
                    mark_phase(3);
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W / 256) : "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                mark_phase(4);
                __syncthreads();
                mark_phase(5);
            }
        } else {
            for (int32_t p = 0; p < nbu; p += U) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int32_t q = p + u;
                    if constexpr (PROF == 1) {
                        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(AE - 1) : "memory");
                        mark_phase(0);
                    }
                    finish(read(xs[u % 3], E[u % AE]));
                    if constexpr (PROF == 1) {
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        mark_phase(1);
                    }
                    E[u % AE] = load_e(q + AE);
                    if (q < nb) __syncthreads();
                    mark_phase(2);
                }
            }
        }
    } else {
        for (int32_t p = 0; p < nbu; p += U) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int32_t q = p + u;
                if (q + AX >= cw + 64) advance();
                load_x(q + AX, X[u % AX]);
                const RState st = read(xs[u & 1], E[u % AE]);
                store_x((u + 1) & 1, X[(u + 1) % AX]);
                finish(st);
                E[u % AE] = load_e(q + AE);
                if (q < nb) __syncthreads();
            }
        }
    }
#ifdef SM_DEV
    if constexpr (PROF == 2) {
        if (threadIdx.x == 0 && blockIdx.x < 4096) g_b2_ts[kTs * blockIdx.x + 1] = wall_clock64();
    }
#endif

    auto flush_prof = [&]() {
#ifdef SM_DEV
        if constexpr (PROF == 2) {
            if (threadIdx.x == 0 && blockIdx.x < 4096) g_b2_ts[kTs * blockIdx.x + 2] = wall_clock64();
        }
        if constexpr (PROF == 1) {   // [6] bands, [7] applying waves (the loader adds 1 << 32)
            ph[6] = (unsigned long long)nb;
            ph[7] = wid == kLdWave ? (1ull << 32) : 1ull;
            if (lane == 0)
                for (int k = 0; k < 8; ++k) atomicAdd(&g_b2_prof[k], ph[k]);
        }
#endif
    };
    if (n_slabs == 1) {
        const int32_t nv = y_vec ? (nr & ~3) : 0;   // float4 rows, then the rest
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int32_t i = 4 * (tid + q * kB2Threads);
            if (i < nv) *reinterpret_cast<float4 *>(y + r0 + i) = *reinterpret_cast<const float4 *>(&yacc[i]);
        }
        for (int32_t i = nv + tid; i < nr; i += kB2Threads) y[r0 + i] = yacc[i];
        flush_prof();
        return;
    }
    __syncthreads();   // every wave is past its last x read: the hand-off words live there
    int32_t *s_word = reinterpret_cast<int32_t *>(&xs[0][0]);
    unsigned long long *ts = nullptr;
#ifdef SM_DEV
    if constexpr (PROF == 2) {
        if (blockIdx.x < 4096) ts = &g_b2_ts[kTs * blockIdx.x + 3];
    }
#endif
    slab_handoff_epoch<kB2Threads, SM_B2_BL != 0>(yacc, ctl + (int64_t)b * kCtlWords, s_word, y, partials,
                                                  n_rows, r0, nr, slab, n_slabs, y_vec, old_started, snap, beta,
                                                  ts);
    flush_prof();
}

#ifdef SM_DEV
// Development read-out of PROF 1 / 2 (tools/cband_prof.py).
template <int GEO>
hipError_t launch_prof(int prof, dim3 grid, hipStream_t s, const XbandDev &xb, int32_t n_rows, int32_t n_cols,
                       const float *x, float *y, float alpha, float beta) {
#define SM_B2P(P)                                                                                   \
    hipLaunchKernelGGL((spmv_band2_kernel<true, GEO, P>), grid, dim3(kB2Threads), 0, s, n_rows, n_cols, \
                       xb.block_rows, xb.n_slabs, xb.d_chunk_start, xb.d_band_clo, xb.d_word,          \
                       xb.d_table, xb.table_size, x, y, xb.d_partials, xb.d_tickets, alpha, beta)
    if (prof == 1) {
        if (GEO != 4) return hipErrorInvalidValue;
        unsigned long long h[8] = {};
        void *sym = nullptr;
        if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_b2_prof)) != hipSuccess) return hipErrorInvalidValue;
        (void)hipMemsetAsync(sym, 0, sizeof(h), s);
        SM_B2P(1);
        (void)hipMemcpyAsync(h, sym, sizeof(h), hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        const double wa = (double)(h[7] & 0xFFFFFFFFull), wl = (double)(h[7] >> 32);
        const double bands = (double)h[6] / (wa + wl);
        fprintf(stderr, "dma3 prof (cycles per band per wave; %.0f applying + %.0f loader waves, %.1f bands): "
                "apply waves: entry wait %.0f apply %.0f barrier %.0f | loader: issue %.0f dma wait %.0f "
                "barrier %.0f\n", wa, wl, bands, h[0] / wa / bands, h[1] / wa / bands, h[2] / wa / bands,
                h[3] / wl / bands, h[4] / wl / bands, h[5] / wl / bands);
        return hipGetLastError();
    }
    const int nt = (int)std::min<int64_t>(grid.x, 4096);
    std::vector<unsigned long long> h((size_t)kTs * nt);
    void *sym = nullptr;
    if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_b2_ts)) != hipSuccess) return hipErrorInvalidValue;
    (void)hipMemsetAsync(sym, 0, h.size() * 8, s);
    SM_B2P(2);
#undef SM_B2P
    (void)hipMemcpyAsync(h.data(), sym, h.size() * 8, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    unsigned long long t0 = ~0ull;
    for (int i = 0; i < nt; i++) t0 = std::min(t0, h[kTs * i]);
    // us (100 MHz): start, loop, epilogue, end; the hand-off's phases where it ran (several slabs)
    std::vector<double> st(nt), lp(nt), ep(nt), en(nt), pb(nt), ad(nt), pl(nt), cb(nt);
    const bool ho = xb.n_slabs > 1;
    for (int i = 0; i < nt; i++) {
        const unsigned long long *u = &h[(size_t)kTs * i];
        st[i] = (u[0] - t0) * 0.01;
        lp[i] = (u[1] - u[0]) * 0.01;
        ep[i] = (u[2] - u[1]) * 0.01;
        en[i] = (u[2] - t0) * 0.01;
        if (ho) {
            pb[i] = (u[3] - u[1]) * 0.01;
            ad[i] = (u[4] - u[3]) * 0.01;
            pl[i] = (u[5] - u[4]) * 0.01;
            cb[i] = (u[6] - u[5]) * 0.01;
        }
    }
    auto pr = [](const char *nm, std::vector<double> v) {
        std::sort(v.begin(), v.end());
        const size_t k = v.size();
        fprintf(stderr, "  %-9s min %6.2f p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us\n", nm, v[0], v[k / 10],
                v[k / 2], v[9 * k / 10], v[k - 1]);
    };
    fprintf(stderr, "cband tile timeline (%d tiles):\n", nt);
    pr("start", st);
    pr("loop", lp);
    pr("epilogue", ep);
    if (ho) {
        pr(" publish", pb);
        pr(" add", ad);
        pr(" wait", pl);
        pr(" combine", cb);
    }
    pr("end", en);
    if (dev_env("SM_B2_TS_DUMP")) {
        for (int i = 0; i < nt; i++)
            fprintf(stderr, "  tile %4d start %6.2f loop %6.2f epi %6.2f pub %6.2f add %6.2f wait %6.2f comb %6.2f\n",
                    i, st[i], lp[i], ep[i], pb[i], ad[i], pl[i], cb[i]);
    }
    return hipGetLastError();
}
#endif

}  // namespace

hipError_t launch_spmv_band2(const XbandDev &xb, int32_t n_rows, int32_t n_cols, const float *x,
                             float *y, float alpha, float beta, hipStream_t s) {
    if (xb.n_blocks <= 0) return hipSuccess;
    const bool cb = xb.kind == kXbCband;
    const bool dma3 = xb.band_cols == kB2Dma3Cb.window;   // cband or band2 entries
    const B2Geom g = dma3 ? (cb ? kB2Dma3Cb : kB2Dma3B2) : kB2Wide;
    if ((xb.kind != kXbBand2 && !cb) || xb.n_slabs < 1 || xb.block_rows > g.block_rows ||
        xb.band_cols != g.window || !xb.d_chunk_start || !xb.d_band_clo || (xb.n_bands > 0 && !xb.d_word) ||
        (cb && (!xb.d_table || xb.table_size < 0 || xb.table_size > (int32_t)kCbDummyId)) ||
        (xb.n_slabs > 1 && (!xb.d_partials || !xb.d_tickets)))
        return hipErrorInvalidValue;
    const dim3 grid((unsigned)((int64_t)xb.n_blocks * xb.n_slabs));
#ifdef SM_DEV
    static const int prof = [] {
        const char *e = dev_env("SM_BAND2_PROF");
        return e ? atoi(e) : 0;
    }();
    if (prof != 0) {
        if (!cb) return hipErrorInvalidValue;
        return dma3 ? launch_prof<4>(prof, grid, s, xb, n_rows, n_cols, x, y, alpha, beta)
                    : launch_prof<0>(prof, grid, s, xb, n_rows, n_cols, x, y, alpha, beta);
    }
#endif
#define SM_B2(C, T)                                                                                 \
    hipLaunchKernelGGL((spmv_band2_kernel<C, T, 0>), grid, dim3(kB2Threads), 0, s, n_rows, n_cols,    \
                       xb.block_rows, xb.n_slabs, xb.d_chunk_start, xb.d_band_clo, xb.d_word,          \
                       xb.d_table, xb.table_size, x, y, xb.d_partials, xb.d_tickets, alpha, beta)
    if (dma3) {
        if (cb) SM_B2(true, 4); else SM_B2(false, 4);
    } else {
        if (cb) SM_B2(true, 0); else SM_B2(false, 0);
    }
#undef SM_B2
    return hipGetLastError();
}

}  // namespace smamd
