// kernels_band2.hip -- SpMV over the balanced-band layout (band2.cpp, xband.h).
//
// One workgroup (1024 threads, 16 waves) per tile = (block of <= 16384 rows, slab
// of columns), one per CU.  A tile's bands are column windows of <= 8192 columns
// holding exactly 32 chunks of 64 entries (dummies pad the last): wave w applies
// chunks 2w and 2w+1 of every band and gets both with one load per lane -- band2:
// 16 bytes (two words, two fp32 values); cband: 8 bytes (two codebook words, the
// values looked up in an LDS copy of the <= 255-entry table scaled by alpha).
// LDS: two x windows (double-buffered), the block's accumulators (cband: and the
// table).
//
// Per band p, every wave (static register rings, the loop unrolled by 2):
//   load x window p+2 into registers (two float4 per lane),
//   issue band p's LDS reads (x, codebook value, accumulator of each chunk),
//   store x window p+1 (loaded a band ago) into the free LDS buffer -- after the
//   reads, so they do not queue behind 16 waves' stores,
//   finish band p: term = x_lds[col] * (v * alpha), the chunk's terms added to the
//   LDS accumulators in rank rounds (a row's segment runs up consecutive lanes by
//   DPP, its last lane writes; no two lanes touch one row in a round, no atomics),
//   load the entries of band p+2 (into the registers band p's entries held),
//   barrier.
// x goes through registers rather than LDS-DMA: vmcnt retires in issue order, so a
// wave waiting for an LDS-DMA issued this band would also wait for every entry load
// issued before it.  Two bands of lookahead suffice: 4, 6 and 8 measured slower
// (config 2, band2: 38.2 / 39.8 / 41.5 / - us; cband 38.0 / 39.3 / 40.6 / 44.0 us),
// and so did deeper entry-only or x-only lookaheads.
//
// Summation order: bands ascend in column, a row's terms inside a band ascend in
// column (ranks), so inside a tile every row is summed in the reference's order
// (kernel.cc:780-796, per output ascending column); slab 0 starts from beta*y,
// later slabs from -0.0, and the slab sums are added in slab order by the slab
// hand-off (xband_dev.h) -- bit-identical to the reference with one slab, within
// the Sum|terms| bound otherwise, deterministic always.
#include "sm_internal.h"
#include "xband.h"
#include "xband_dev.h"

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <type_traits>

namespace smamd {
namespace {

constexpr int kB2Threads = 1024;
#ifdef SM_DEV
// ABL & 1024 (development builds): lane 0 of every wave adds the cycles (s_memtime) of
// each phase of the band loop here: prologue, x store (its wait), apply, entry load
// issue, barrier, epilogue, bands, waves.
__device__ unsigned long long g_b2_prof[8];
// ABL & 2048: wall clock (s_memrealtime, 100 MHz) of every tile's start, loop end and
// finish, from thread 0.
__device__ unsigned long long g_b2_ts[3 * 4096];
#endif
// Lookaheads (bands) of the x windows and of the entries; development builds
// override them (tools/r2_ab.sh).
#ifndef SM_CB_XAHEAD
#define SM_CB_XAHEAD 2
#endif
#ifndef SM_CB_EAHEAD
#define SM_CB_EAHEAD 2
#endif
// dmaw: entries this many bands ahead (two-buffer windows leave no band of slack for them).
#ifndef SM_CBW_EAHEAD
#define SM_CBW_EAHEAD 4
#endif
#ifndef SM_B2_XAHEAD
#define SM_B2_XAHEAD 2
#endif
#ifndef SM_B2_EAHEAD
#define SM_B2_EAHEAD 2
#endif
// Slab hand-off protocol: 1 = the epoch form (xband_dev.h slab_handoff_epoch: no reset
// round trip at the end, the commit snapshot read behind the band loop), 0 = slab_handoff.
#ifndef SM_B2_EPOCH
#define SM_B2_EPOCH 1
#endif
#ifndef SM_CB_TAB_COPIES
#define SM_CB_TAB_COPIES 32
#endif
// SM_CB_DMA (development A/B, wide cband): x windows go L2 -> LDS by LDS-DMA one
// band ahead (no register ring), entries SM_CB_DMA_EAHEAD bands ahead.
#ifndef SM_CB_DMA
#define SM_CB_DMA 0
#endif
#ifndef SM_CB_DMA_EAHEAD
#define SM_CB_DMA_EAHEAD 4
#endif
#ifndef SM_E_EARLY
#define SM_E_EARLY 0
#endif
#ifndef SM_LD_XPF
#define SM_LD_XPF 0
#endif
#ifndef SM_LD_TPF
#define SM_LD_TPF 0
#endif
#ifndef SM_LD_PRIO
#define SM_LD_PRIO 3
#endif
#ifndef SM_CB_RFIRST
#define SM_CB_RFIRST 1
#endif
#ifndef SM_X_AUX
#define SM_X_AUX 0
#endif
#ifndef SM_ENT_AUX
#define SM_ENT_AUX kAuxNt
#endif
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

// ABL (development only, SM_BAND2_ABLATE; results wrong): 1 skips the apply,
// 2 the x loads and stores, 4 the entry loads, 8 the slab hand-off (plain stores),
// 16 the band loop; cband only: 32 the codebook lookup, 64 the rank rounds, 128
// the x gather (lane-ordered LDS reads instead), 256 the x LDS stores, 512 the
// per-band barrier (racy).
// CB: the cband encoding (xband.h): one 32-bit word per term, values from the
// codebook `table` (<= 255 entries), scaled by alpha once into LDS.
// GEO: the tile geometry (xband.h B2Geom): 0 wide; 1 tall (32K-row blocks, 4096 --
// cband 3840 -- column windows, one float4 of x per lane per band); 2 wide3 (cband:
// 12160-column windows, three chunks per wave per band, the table in one copy).
template <int ABL, int PRIO, bool CB, int GEO>
__global__ __launch_bounds__(kB2Threads) void spmv_band2_kernel(
    int32_t n_rows, int32_t n_cols, int32_t block_rows, int32_t n_slabs,
    const int32_t *__restrict__ tile_band_start, const int32_t *__restrict__ band_clo,
    const uint32_t *__restrict__ ent, const float *__restrict__ table, int32_t table_size,
    const float *__restrict__ x, float *__restrict__ y, float *__restrict__ partials,
    int32_t *__restrict__ ctl, float alpha, float beta, int32_t xcd_map) {
    constexpr bool TALL = GEO == 1;
    static_assert(GEO < 2 || GEO == 4 || CB, "wide3, half2, dma3t and dma3 tall are cband geometries");
    constexpr B2Geom G = TALL ? (CB ? kB2TallCb : kB2TallB2) : GEO == 2 ? kB2Wide3Cb
                       : GEO == 3 ? kB2Half2Cb : GEO == 4 ? (CB ? kB2Dma3Cb : kB2Dma3B2)
                       : GEO == 5 ? kB2Dma3tCb : GEO == 6 ? kB2Dma3TallCb : GEO == 8 ? kB2DmawCb
                       : GEO == 9 ? kB2Dmaw4Cb : kB2Wide;
    static_assert(GEO < 8 || CB, "dmaw is a codebook geometry");
    // dma3: wave kLdWave stages the x windows (LDS-DMA, three buffers, two bands ahead) and
    // the other waves apply -- no x ever passes through an applying wave's registers, and
    // the loader's wait for its DMA is the only vmcnt wait on x (its queue holds nothing else).
    constexpr bool kLd = GEO == 4 || GEO == 5 || GEO == 6 || GEO == 8 || GEO == 9;
    constexpr bool kW = GEO == 8 || GEO == 9;             // dmaw: several loader waves, two x buffers
    constexpr int kNLd = kW ? 16 - G.chunks() / G.cpw : 1;   // loader waves (the last ones)
    constexpr int kLdWave = kB2Threads / 64 - kNLd;       // the first loader wave
    constexpr int CPW = CB ? G.cpw : 2;   // chunks per wave per band
    constexpr int BROWS = G.block_rows;
    constexpr int W = G.window;
    constexpr int XV = (W + 4 * kB2Threads - 1) / (4 * kB2Threads);   // float4 of x per lane
    constexpr int kB2Col = G.col_bits;                                // band2 word fields
    constexpr uint32_t kB2Dummy = G.dummy_word();
    constexpr uint32_t kColMask = (1u << kB2Col) - 1u;
    constexpr uint32_t kRankMask = (1u << kB2RankBits) - 1u;
    // Every LDS byte counts in the tall geometry: band2 keeps per-lane scratch slots
    // for its dummy lanes' writes only in the wide one.
    constexpr bool kScratch = !CB && GEO == 0;
    // Rings: x window p+AX and the entries of band p+AE are loaded at band p into the
    // slots band p just freed (the x of window p was stored a band ago; the entries
    // of band p are loaded after its apply has decoded them).  Waiting for window p+1
    // (loaded AX-1 bands ago) retires every older load.  Measured (config 2): a
    // lookahead of 2 bands beats 6 (38.3 vs 40.6 us cband, 38.3 vs 41.5 band2) --
    // the loads need no more cover, and more of them in flight only slow the rest.
    // kDma: window q+1 is LDS-DMA'd at band q into the buffer band q-1 read; hipcc
    // does not count the (asm) DMA, so its own wait for the entries of band q counts
    // only the AE-1 younger entry loads -- at least the 3 ops really pending then
    // (one entry load, the window's two DMA pieces) once AE >= 4: no extra stall.
    constexpr bool kDma = CB && GEO == 0 && SM_CB_DMA != 0;
    constexpr int kXBuf = kLd && !kW ? 3 : 2;   // x window buffers in LDS
    static_assert(!kDma || SM_CB_DMA_EAHEAD >= 4, "DMA variant: hipcc's entry waits must not stall");
    constexpr int AX = kDma ? 1 : CB ? SM_CB_XAHEAD : SM_B2_XAHEAD;
    // XPF (dma3 + codebook, SM_LD_XPF): band q+1's x and codebook values are read during band q,
    // once the loader has flagged window q+1 in LDS, so after each barrier only the accumulator
    // reads queue; its entries come 3 bands ahead (band q+1's must be in registers by then).
    constexpr bool kXpf = kLd && CB && SM_LD_XPF != 0;
    constexpr int AE = kW ? SM_CBW_EAHEAD : kXpf ? 3 : kDma ? SM_CB_DMA_EAHEAD : CB ? SM_CB_EAHEAD : SM_B2_EAHEAD;
    // SM_E_EARLY (development A/B): the entries of band p+AE are loaded before band p's
    // apply into a ring of AE+1 slots (the slot of band p-1 is free by then).
    constexpr bool kEarly = SM_E_EARLY != 0;
    // cband: the apply's LDS reads go out before the next x window's LDS stores, so
    // they do not queue behind 16 waves' stores (config 2: 37.1 vs 39.6 us with the
    // stores first; SM_CB_RFIRST=0 restores that order in development builds).
    constexpr bool kRFirst = !kDma && !kEarly && SM_CB_RFIRST != 0 && !(ABL & 1);
    constexpr int ER = kEarly ? AE + 1 : AE;   // entry ring slots
    constexpr int U0 = AX > ER ? AX : ER;
    constexpr int UA = U0 % 2 ? 2 * U0 : (U0 % AX ? U0 * AX : U0);   // loop unroll: static roles
    constexpr int U = kW ? (ER % 2 ? 2 * ER : ER) : kLd ? (ER % 3 == 0 ? 2 * ER : 6 * ER / (ER % 2 ? 1 : 2)) : UA;
    static_assert(U % AX == 0 && U % ER == 0 && U % 2 == 0 && (!kLd || U % kXBuf == 0), "ring sizes divide the unroll");
    static_assert(W % 4 == 0 && XV * 4 * kB2Threads >= W, "float4 slots cover the window");
    __shared__ __attribute__((aligned(16))) float xs[kXBuf][W];
    // Wide band2: + a scratch slot per lane (dummy lanes write there).  The other
    // kinds write only live lanes and use the LDS nearly to the last byte: their
    // hand-off words live in the x buffers once the band loop is over.
    __shared__ __attribute__((aligned(16))) float yacc[BROWS + (kScratch ? 64 : 0)];
    // cband: fl(table[id] * alpha) (0 past the table) in kTabCopies copies, entry id
    // of copy c at kTabCopies * id + c: lane l reads copy l % kTabCopies, so the
    // reads of a 32-lane group spread over the banks whatever the ids (wide: 32
    // copies, every group conflict-free -- 37.3 vs 38.1 us with 16, 39.1 with 8,
    // 38.6 with 4 on config 2; tall: one, no room for more).
    constexpr int kTabCopies = GEO == 0 ? SM_CB_TAB_COPIES : G.tab_copies;
    __shared__ float tab[CB ? 256 * kTabCopies : 1];
    __shared__ int32_t s_xready;   // XPF: the highest window the loader has seen land
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    constexpr bool kProf = (ABL & 1024) != 0 && !kLd;
    // dma3 (ABL & 4096, development): cycles per band of every phase -- applying waves: the
    // entry wait, the apply, the barrier; the loader: the DMA issue, its wait, the barrier.
    constexpr bool kProfLd = (ABL & 4096) != 0 && kLd;
    [[maybe_unused]] constexpr bool kTs = (ABL & 2048) != 0;
#ifdef SM_DEV
    if constexpr (kTs) {
        if (threadIdx.x == 0 && blockIdx.x < 4096) g_b2_ts[3 * blockIdx.x] = wall_clock64();
    }
#endif
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tk = (kProf || kProfLd) ? clock64() : 0;
    auto mark_phase = [&](int k) {
        if constexpr (kProf || kProfLd) {
            const unsigned long long now = clock64();
            ph[k] += now - tk;
            tk = now;
        }
    };
    // Tile of this workgroup.  xcd_map: workgroup i runs on XCD i % 8 (dispatch round
    // robin), so tile = the i / 8-th of XCD (i % 8)'s contiguous range of tiles: the
    // slabs of one row block share an XCD and their hand-off stays in its L2.
    int32_t t = blockIdx.x;
    if (xcd_map == 1) {
        const int32_t G = gridDim.x, xc = t & 7, k = t >> 3;
        t = xc * (G >> 3) + min(xc, G & 7) + k;
    } else if (xcd_map == 2 && n_slabs == 4 && gridDim.x == 256) {
        // XCD pairs (development A/B): XCDs 2j and 2j+1 hold the blocks b = j (mod 4), slabs
        // 0-1 on the first and 2-3 on the second -- two slabs of x per L2, and each
        // block's hand-off crosses the fabric between two XCDs instead of four.
        const int32_t xc = t & 7, k = t >> 3;
        const int32_t b2 = (xc >> 1) + 4 * (k >> 1);
        t = 4 * b2 + 2 * (xc & 1) + (k & 1);
    }
    const int32_t b = t / n_slabs;
    const int32_t slab = t - b * n_slabs;
#if SM_B2_EPOCH
    const uint64_t old_started = (ABL & 8) ? 0u : handoff_begin(ctl + (int64_t)b * kCtlWords, n_slabs);
#else
    if (!(ABL & 8)) handoff_started(ctl + (int64_t)b * kCtlWords, n_slabs);
#endif
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
    // Band windows: lane l holds clo of bands cw + l (lo) and cw + 64 + l (hi), read
    // by readlane; the window advances by 64 bands when the x loads reach its hi half.
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

    // x window q: float4 slots tid (+ 1024) of [clo_q, clo_q + W); windows past the
    // tile and slots past W read nothing (offset past the descriptor).
    auto load_x = [&](int32_t q, float4 *xr) {
        const int32_t c = q < nb ? clo_at(q) : 0;
#pragma unroll
        for (int k = 0; k < XV; ++k) {
            const int32_t slot = 4 * (tid + k * kB2Threads);
            const uint32_t off = q < nb && slot < W ? 4u * (uint32_t)(c + slot) : 0xFFFFFFF0u;
            u32x4 v = {off, off, off, off};
            if (!(ABL & 2)) v = __builtin_amdgcn_raw_buffer_load_b128(x_src, off, 0, SM_X_AUX);
            xr[k] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                                __uint_as_float(v.w));
        }
    };
    // kDma: piece m (256 floats, 1 KiB) of window q is wave-instruction k of wave
    // m % 16; windows past the tile land zeros in a buffer nobody reads any more.
    const uint32_t xs_lds = (uint32_t)(size_t)(__attribute__((address_space(3))) float *)&xs[0][0];
    auto dma_x = [&](int32_t q, int buf) {
        const int32_t c = q < nb ? clo_at(q) : 0;
#pragma unroll
        for (int k = 0; k < XV; ++k) {
            const int32_t m = k * (kB2Threads / 64) + (tid >> 6);
            const uint32_t voff =
                q < nb && !(ABL & 2) ? 4u * (uint32_t)(c + m * 256 + lane * 4) : 0xFFFFFFF0u;
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
    // dma3: the loader wave's LDS-DMA of window q into buffer buf, W / 256 pieces of 1 KiB
    // (one wave-instruction each); only windows of the tile are issued.
    auto wid_ld = [&]() { return (int)__builtin_amdgcn_readfirstlane(tid >> 6) - kLdWave; };
    constexpr int kPieces = W / 256;
    constexpr int kPpl = (kPieces + kNLd - 1) / kNLd;   // pieces per loader wave
    auto dma_win = [&](int32_t c, int32_t buf) {   // c: the window's first column
        const int ld = kNLd > 1 ? wid_ld() : 0;
#pragma unroll
        for (int k = 0; k < kPpl; ++k) {
            const int m = ld + k * kNLd;
            if (kPieces % kNLd != 0 && m >= kPieces) break;   // wave-uniform
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
    static_assert(!kLd || W % 256 == 0, "dma3 windows are whole 1 KiB pieces");
    auto store_x = [&](int buf, const float4 *xr) {
#pragma unroll
        for (int k = 0; k < XV; ++k) {
            const int32_t slot = 4 * (tid + k * kB2Threads);
            if (ABL & (2 | 256))
                asm volatile("" ::"v"(xr[k].x), "v"(xr[k].y), "v"(xr[k].z), "v"(xr[k].w));
            else if (W % (4 * kB2Threads) == 0 || slot < W)
                *reinterpret_cast<float4 *>(&xs[buf][slot]) = xr[k];
        }
    };
    // Entries of band q: band2 {word 2w, word 2w+1, value 2w, value 2w+1}, cband
    // {word 2w, word 2w+1} for this lane; past the tile: zeros = dummies.
    using EV = typename std::conditional<
        CB, typename std::conditional<CPW == 6, u32x8,
                typename std::conditional<CPW == 4, u32x4,
                        typename std::conditional<CPW == 3, u32x3, u32x2>::type>::type>::type,
        u32x4>::type;
    auto load_e = [&](int32_t q) -> EV {
        const uint32_t off = (kApplyThreads < kB2Threads && tid >= kApplyThreads)
                                 ? 0xFFFFFFF0u
                                 : kBandBytes * (uint32_t)q + (kBandBytes / kApplyThreads) * (uint32_t)tid;
        if (ABL & 4) return EV{};
        if constexpr (CB && CPW == 6) {   // 24 bytes per lane: 16 + 8
            const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(e_src, off, 0, SM_ENT_AUX);
            const u32x2 b = __builtin_amdgcn_raw_buffer_load_b64(e_src, off >= 0xFFFFFFF0u ? off : off + 16u, 0,
                                                                 SM_ENT_AUX);
            EV r;
            r.s0 = a.x; r.s1 = a.y; r.s2 = a.z; r.s3 = a.w; r.s4 = b.x; r.s5 = b.y; r.s6 = 0u; r.s7 = 0u;
            return r;
        } else if constexpr (CB && CPW == 4) {
            return __builtin_amdgcn_raw_buffer_load_b128(e_src, off, 0, SM_ENT_AUX);
        } else if constexpr (CB && CPW == 3)
            return __builtin_amdgcn_raw_buffer_load_b96(e_src, off, 0, SM_ENT_AUX);
        else if constexpr (CB)
            return __builtin_amdgcn_raw_buffer_load_b64(e_src, off, 0, SM_ENT_AUX);
        else
            return __builtin_amdgcn_raw_buffer_load_b128(e_src, off, 0, SM_ENT_AUX);
    };

    auto shr1 = [](float v) {   // lane i <- lane i-1 (lane 0 never has rank >= 1)
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, false));
    };
    auto shl1 = [](uint32_t v) {   // lane i <- lane i+1; lane 63 <- the dummy rank
        return (uint32_t)__builtin_amdgcn_update_dpp((int)kB2DummyRank, (int)v, 0x130, 0xF, 0xF, false);
    };
    (void)kB2Dummy;
    // band2 apply in two steps like cband's (b2_read issues the four LDS reads, the
    // loop stores the next x window, b2_finish adds and writes).
    struct B2State {
        float xv[2], yv[2], va[2];
        uint32_t rk[2], rl[2];
        bool live[2];
        bool more;
    };
    auto b2_read = [&](const float *xb, u32x4 e) -> B2State {
        if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(PRIO);
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
        if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(0);
    };
    auto apply_b2 = [&](const float *xb, u32x4 e) { b2_finish(b2_read(xb, e)); };

    // Lane select by an SGPR lane mask (v_cndmask_b32 with the mask as its condition):
    // lane i takes b where bit i of m is set, else a.
    auto sel = [](uint64_t m, float a, float b) -> float {
        float r;
        asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
        return r;
    };
    // cband: row = chunk base (lane 0's header) + offset.  A segment's running sum
    // moves up one lane per round in lane (= column) order; the lanes a round updates
    // are an SGPR mask: the continuations whose predecessor finished last round.
    // Two steps: cb_read decodes the chunk words and issues the 3 * CPW LDS reads,
    // cb_finish adds and writes; the loop puts the next x window's LDS stores between
    // them so the reads do not queue behind 16 waves' stores.
    constexpr uint32_t kCbCol = (1u << G.cb_col) - 1u;
    constexpr uint32_t kCbDummy = G.cb_dummy_word();
    constexpr int kCbOffSh = G.cb_off_shift();
    constexpr uint32_t kCbOffM = G.cb_off_mask();
    struct CbState {
        float xv[CPW], yv[CPW], tv[CPW];
        uint32_t rl[CPW];
        uint64_t live[CPW], cont[CPW];
    };
    // The codebook values of a band's two chunks (dma3 reads them a band early, TPF).
    auto tab_read = [&](EV e, float *tv) {
#pragma unroll
        for (int k = 0; k < CPW; ++k) {
            const uint32_t id = ((e[k] ^ kCbDummy) >> G.cb_col) & kCbDummyId;
            tv[k] = tab[id * kTabCopies + (lane & (kTabCopies - 1))];
        }
    };
    auto cb_read = [&](const float *xb, EV e, const float *tv_pre = nullptr,
                       const float *xv_pre = nullptr) -> CbState {
        if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(PRIO);
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
            st.xv[k] = xv_pre ? xv_pre[k] : xb[(ABL & 128) ? (uint32_t)(lane + 64 * k) : (wd & kCbCol)];
            st.tv[k] = (ABL & 32) ? __uint_as_float(id)
                       : tv_pre ? tv_pre[k] : tab[id * kTabCopies + (lane & (kTabCopies - 1))];
            st.yv[k] = yacc[st.rl[k]];
        }
        return st;
    };
    auto cb_finish = [&](CbState st) {
        float *xv = st.xv, *yv = st.yv, *tv = st.tv;
        // Materialise all reads before any write (one LDS wait per band).
        if constexpr (CPW > 3) {
#pragma unroll
            for (int k = 0; k < CPW; ++k) asm volatile("" : "+v"(xv[k]), "+v"(yv[k]), "+v"(tv[k]));
        } else if constexpr (CPW == 3)
            asm volatile("" : "+v"(xv[0]), "+v"(xv[1]), "+v"(xv[2]), "+v"(yv[0]), "+v"(yv[1]), "+v"(yv[2]),
                         "+v"(tv[0]), "+v"(tv[1]), "+v"(tv[2]));
        else
            asm volatile("" : "+v"(xv[0]), "+v"(xv[1]), "+v"(yv[0]), "+v"(yv[1]), "+v"(tv[0]), "+v"(tv[1]));
        float tm[CPW], acc[CPW];
        uint64_t R[CPW];
#pragma unroll
        for (int k = 0; k < CPW; ++k) {
            tm[k] = __fmul_rn(xv[k], tv[k]);
            acc[k] = __fadd_rn(yv[k], tm[k]);
            R[k] = st.cont[k] & ~(st.cont[k] << 1);
        }
        if constexpr (!(ABL & 64)) {
            auto any = [&]() {
                uint64_t a = 0;
#pragma unroll
                for (int k = 0; k < CPW; ++k) a |= R[k];
                return a != 0;
            };
            while (any()) {
#pragma unroll
                for (int k = 0; k < CPW; ++k) {
                    acc[k] = sel(R[k], acc[k], __fadd_rn(shr1(acc[k]), tm[k]));
                    R[k] = st.cont[k] & (R[k] << 1);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < CPW; ++k) {   // the segment's last lane writes its row
            const uint64_t last = st.live[k] & ~(st.cont[k] >> 1);
            if ((last >> lane) & 1) yacc[st.rl[k]] = acc[k];
        }
        if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(0);
    };
    auto apply_cb = [&](const float *xb, EV e) { cb_finish(cb_read(xb, e)); };

    // Prologue, ordered so its memory latencies overlap: the first windows' x and entry
    // loads go out first, then the codebook and (slab 0) y loads; the LDS writes of all
    // of them follow, so the tile waits about one memory latency before its first band
    // instead of one per kind of load (vmcnt retires in issue order).
    // Rings with static roles: x window q in X[q % AX], entries of band q in E[q % AE].
    // Prologue = virtual bands -U..-1 (their loads in the loop's order), so the loads
    // pending at the loop header are in the order the loop's back edge leaves them.
    float4 X[AX][XV];
    EV E[ER];
    const int32_t wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR)
    if constexpr (kLd) {
#pragma unroll
        for (int v = 0; v < AE; ++v) E[v] = load_e(v);
        if (wid >= kLdWave) {   // windows 0 and 1 (dmaw: 0); waited for (with everything) below
            if (nb > 0) dma_win(clg[0], 0);
            if (!kW && nb > 1) dma_win(clg[1], 1);
        }
    } else if constexpr (kDma) {
#pragma unroll
        for (int v = 0; v < AE; ++v) E[v] = load_e(v);
        dma_x(0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
#pragma unroll
        for (int v = -U; v < 0; ++v) {
            if (v + AX >= 0) load_x(v + AX, X[v + AX]);
            if (v + AE >= 0) E[(v + AE) % ER] = load_e(v + AE);
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
    // Accumulators: beta*y (slab 0) or -0.0 (the identity of fp32 addition: a row
    // without terms in this slab keeps the sign of a zero y), all loads in flight.
    constexpr int kQ = BROWS / (4 * kB2Threads);
    const bool y_vec = ((uintptr_t)(y + r0) & 15) == 0;
    float4 yv[kQ];
    if (slab == 0) {
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
    if (slab == 0) {
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
        if (wid >= kLdWave) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if constexpr (kXpf)
                if (lane == 0) __hip_atomic_store(&s_xready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    } else if constexpr (!kDma) {
        store_x(0, X[0]);
    }
    __syncthreads();
#if SM_B2_EPOCH
    // The commit check's snapshot (xband_dev.h slab_handoff_epoch): read now, used after the
    // band loop, so its round trip hides behind the loop.
    const uint64_t snap = (ABL & 8) ? 0u : handoff_snapshot(ctl + (int64_t)b * kCtlWords, n_slabs);
#endif

    // Whole groups of U bands (static ring indices, no branch around a load or a
    // ring register: either makes hipcc copy registers and drain vmcnt).  Steps past
    // the tile's last band see only dummy entries (their loads go past the
    // descriptors: no memory request) and skip the barrier -- a uniform branch; the
    // dummies write nothing but the x buffers nobody reads any more (band2: and the
    // scratch slots).
    const int32_t nbu = (ABL & 16) ? 0 : (nb + U - 1) / U * U;
    mark_phase(0);
    if constexpr (kProfLd) ph[0] = 0;   // the prologue is not a band phase
    if constexpr (kW) {
        if (wid >= kLdWave) {
            // dmaw, band q: window q+1 into the buffer window q-1 left (every wave passed band
            // q-1's barrier), wait until this wave's pieces of it have landed, meet the others
            // at the barrier.  The windows' first columns come by scalar loads one band ahead.
            int32_t c_next = nb > 1 ? clg[1] : 0;
            __builtin_amdgcn_s_setprio(SM_LD_PRIO);
            for (int32_t q = 0; q < nb; ++q) {
                if (q + 1 < nb) {
                    const int32_t c = c_next;
                    const int32_t qn = __builtin_amdgcn_readfirstlane(q + 2);
                    if (qn < nb) c_next = clg[qn];
                    if constexpr (kProfLd) mark_phase(5);
                    dma_win(c, (q + 1) & 1);
                    if constexpr (kProfLd) mark_phase(3);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if constexpr (kProfLd) mark_phase(4);
                if constexpr (!(ABL & 512)) __syncthreads();
                if constexpr (kProfLd) mark_phase(5);
            }
        } else {
            for (int32_t p = 0; p < nbu; p += U) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int32_t q = p + u;
                    if constexpr (kProfLd) {
                        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((CPW == 6 ? 2 : 1) * (AE - 1)) : "memory");
                        mark_phase(0);
                    }
                    if constexpr (ABL & 1) {
                        asm volatile("" ::"v"(E[u % ER].s0), "v"(E[u % ER].s1));
                    } else {
                        apply_cb(xs[u % kXBuf], E[u % ER]);
                    }
                    if constexpr (kProfLd) {
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        mark_phase(1);
                    }
                    E[u % ER] = load_e(q + AE);
                    if (!(ABL & 512) && q < nb) __syncthreads();
                    if constexpr (kProfLd) mark_phase(2);
                }
            }
        }
    } else if constexpr (kLd) {
        if (wid == kLdWave) {
            // Band q: DMA window q+2 into the buffer window q-1 left (every wave passed
            // band q-1's barrier), then wait until window q+1 has landed -- the 30 pieces
            // just issued may stay in flight -- and meet the others at the barrier.
            // The windows' first columns come by scalar loads one band ahead (a vector load
            // here would make hipcc wait for the whole DMA queue before reading it).
            int32_t c_next = nb > 2 ? clg[2] : 0;
            __builtin_amdgcn_s_setprio(SM_LD_PRIO);   // the DMA issue goes first
            for (int32_t q = 0; q < nb; ++q) {
                if (q + 2 < nb) {
                    const int32_t c = c_next;
                    const int32_t qn = __builtin_amdgcn_readfirstlane(q + 3);
                    if (qn < nb) c_next = clg[qn];
                    if constexpr (kProfLd) mark_phase(5);
                    dma_win(c, (q + 2) % 3);
                    if constexpr (kProfLd) mark_phase(3);
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W / 256) : "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if constexpr (kXpf)   // window q+1 has landed: the appliers may read it now
                    if (lane == 0) __hip_atomic_store(&s_xready, q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if constexpr (kProfLd) mark_phase(4);
                if constexpr (!(ABL & 512)) __syncthreads();   // 512: no band barriers (racy, A/B)
                if constexpr (kProfLd) mark_phase(5);
            }
        } else {
            // TPF (SM_LD_TPF=1, development A/B): band q+1's codebook values read during band q,
            // so after each barrier only the x and accumulator reads queue on the LDS -- measured
            // slower (35.5 vs 34.1 us: its wait for band q+1's entries, one band after their load).
            constexpr bool kTpf = SM_LD_TPF != 0 && CB && !kXpf;
            float tvn[CPW];
            if constexpr (kTpf) tab_read(E[0], tvn);
            float xpv[CPW], xpt[CPW];   // XPF: band q's x and codebook values, read during band q-1
            auto xpf_read = [&](const float *xb, EV e) {
#pragma unroll
                for (int k = 0; k < CPW; ++k) {
                    const uint32_t wd = e[k] ^ kCbDummy;
                    const uint32_t id = (wd >> G.cb_col) & kCbDummyId;
                    xpv[k] = xb[wd & kCbCol];
                    xpt[k] = tab[id * kTabCopies + (lane & (kTabCopies - 1))];
                }
            };
            if constexpr (kXpf) xpf_read(xs[0], E[0]);   // window 0 landed before the prologue barrier
            for (int32_t p = 0; p < nbu; p += U) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int32_t q = p + u;
                    if constexpr (kProfLd) {
                        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(AE - 1) : "memory");
                        mark_phase(0);
                    }
                    if constexpr (ABL & 1) {
                        asm volatile("" ::"v"(E[u % ER].x), "v"(E[u % ER].y));
                    } else if constexpr (!CB) {
                        apply_b2(xs[u % 3], E[u % ER]);
                    } else if constexpr (kXpf) {
                        CbState st = cb_read(xs[u % 3], E[u % ER], xpt, xpv);
                        cb_finish(st);
                        if (q + 1 < nb) {   // band q+1's window flagged, then its x and codebook reads
                            while (__hip_atomic_load(&s_xready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < q + 1)
                                __builtin_amdgcn_s_sleep(1);
                            xpf_read(xs[(u + 1) % 3], E[(u + 1) % ER]);
                        }
                    } else if constexpr (kTpf) {
                        // band q's reads, then band q+1's codebook reads behind them (they
                        // land while band q adds), then band q's adds and writes
                        const CbState st = cb_read(xs[u % 3], E[u % ER], tvn);
                        asm volatile("" ::: "memory");   // keep band q's reads first in the LDS queue
                        tab_read(E[(u + 1) % ER], tvn);
                        cb_finish(st);
                    } else {
                        apply_cb(xs[u % 3], E[u % ER]);
                    }
                    if constexpr (kProfLd) {
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        mark_phase(1);
                    }
                    E[u % ER] = load_e(q + AE);
                    if (!(ABL & 512) && q < nb) __syncthreads();
                    if constexpr (kProfLd) mark_phase(2);
                }
            }
        }
    } else
    for (int32_t p = 0; p < nbu; p += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t q = p + u;
            if (q + AX >= cw + 64) advance();
            using RState = typename std::conditional<CB, CbState, B2State>::type;
            [[maybe_unused]] RState st_rf;
            if constexpr (kDma) {
                dma_x(q + 1, (u + 1) & 1);
            } else if constexpr (kRFirst) {
                load_x(q + AX, X[u % AX]);
                if constexpr (CB) st_rf = cb_read(xs[u & 1], E[u % ER]);
                else st_rf = b2_read(xs[u & 1], E[u % ER]);
                store_x((u + 1) & 1, X[(u + 1) % AX]);
            } else {
                load_x(q + AX, X[u % AX]);
                store_x((u + 1) & 1, X[(u + 1) % AX]);
            }
            if constexpr (kProf) {   // the x store's wait, made visible
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                mark_phase(1);
            }
            if constexpr (kEarly) E[(u + AE) % ER] = load_e(q + AE);
            if constexpr (ABL & 1) {
                asm volatile("" ::"v"(E[u % ER].x), "v"(E[u % ER].y));
            } else if constexpr (kRFirst) {
                if constexpr (CB) cb_finish(st_rf);
                else b2_finish(st_rf);
            } else if constexpr (CB) {
                apply_cb(xs[u & 1], E[u % ER]);
            } else {
                apply_b2(xs[u & 1], E[u % ER]);
            }
            if constexpr (kProf) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                mark_phase(2);
            }
            if constexpr (!kEarly) E[u % ER] = load_e(q + AE);
            mark_phase(3);
            // kDma: window q+1 landed (in-order retirement); the entry load just issued flies.
            if constexpr (kDma) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
            if (!(ABL & 512) && q < nb) __syncthreads();
            mark_phase(4);
        }
    }
    if constexpr (kProf) {
        ph[6] = (unsigned long long)nb;
        ph[7] = 1;
    }
#ifdef SM_DEV
    if constexpr (kTs) {
        if (threadIdx.x == 0 && blockIdx.x < 4096) g_b2_ts[3 * blockIdx.x + 1] = wall_clock64();
    }
#endif

    auto flush_prof = [&]() {
#ifdef SM_DEV
        if constexpr (kTs) {
            if (threadIdx.x == 0 && blockIdx.x < 4096) g_b2_ts[3 * blockIdx.x + 2] = wall_clock64();
        }
        if constexpr (kProf) {
            mark_phase(5);
            if (lane == 0)
                for (int k = 0; k < 8; ++k) atomicAdd(&g_b2_prof[k], ph[k]);
        }
        if constexpr (kProfLd) {   // [6] bands, [7] applying waves (the loader adds 1 << 32)
            ph[6] = (unsigned long long)nb;
            ph[7] = wid >= kLdWave ? (1ull << 32) : 1ull;
            if (lane == 0)
                for (int k = 0; k < 8; ++k) atomicAdd(&g_b2_prof[k], ph[k]);
        }
#endif
    };
    if (n_slabs == 1 || (ABL & 8)) {
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
#if SM_B2_EPOCH
    slab_handoff_epoch<kB2Threads>(yacc, ctl + (int64_t)b * kCtlWords, s_word, y, partials, n_rows, r0,
                                   nr, slab, n_slabs, y_vec, old_started, snap);
#else
    slab_handoff<kB2Threads>(yacc, ctl + (int64_t)b * kCtlWords, s_word, y, partials, n_rows, r0,
                             nr, slab, n_slabs, y_vec);
#endif
    flush_prof();
}

}  // namespace

hipError_t launch_spmv_band2(const XbandDev &xb, int32_t n_rows, int32_t n_cols, const float *x,
                             float *y, float alpha, float beta, hipStream_t s) {
    if (xb.n_blocks <= 0) return hipSuccess;
    const bool cb = xb.kind == kXbCband;
    const bool wide3 = cb && xb.band_cols == kB2Wide3Cb.window;
    const bool half2 = cb && xb.band_cols == kB2Half2Cb.window;
    const bool dma3 = xb.band_cols == kB2Dma3Cb.window;   // cband or band2 entries
    const bool dma3t = cb && xb.band_cols == kB2Dma3tCb.window;
    const bool dma3tall = cb && xb.band_cols == kB2Dma3TallCb.window;
    const bool dmaw_any = cb && xb.band_cols == kB2DmawCb.window;
    const bool dmaw4 = dmaw_any && xb.kind == kXbCband && xb.chunks_per_wave == 4;
    const bool dmaw = dmaw_any && !dmaw4;
    const bool tall = !wide3 && !half2 && !dma3 && !dma3t && !dma3tall && !dmaw_any && xb.band_cols != kB2Wide.window;
    const B2Geom g = wide3 ? kB2Wide3Cb : half2 ? kB2Half2Cb : dma3 ? (cb ? kB2Dma3Cb : kB2Dma3B2) : dma3t ? kB2Dma3tCb
                   : dma3tall ? kB2Dma3TallCb : dmaw ? kB2DmawCb : dmaw4 ? kB2Dmaw4Cb : tall ? (cb ? kB2TallCb : kB2TallB2) : kB2Wide;
    if ((xb.kind != kXbBand2 && !cb) || xb.n_slabs < 1 || xb.block_rows > g.block_rows ||
        xb.band_cols != g.window || !xb.d_chunk_start || !xb.d_band_clo ||
        (xb.n_bands > 0 && !xb.d_word) ||
        (cb && (!xb.d_table || xb.table_size < 0 || xb.table_size > (int32_t)kCbDummyId)) ||
        (xb.n_slabs > 1 && (!xb.d_partials || !xb.d_tickets)))
        return hipErrorInvalidValue;
    const dim3 grid((unsigned)((int64_t)xb.n_blocks * xb.n_slabs)), block(kB2Threads);
    int32_t xcd_map = 0;
#ifdef SM_DEV
    if (const char *e = dev_env("SM_B2_XCDMAP")) xcd_map = atoi(e);
#endif
#define SM_B2(A, P, C, T)                                                                      \
    hipLaunchKernelGGL((spmv_band2_kernel<A, P, C, T>), grid, block, 0, s, n_rows, n_cols,    \
                       xb.block_rows, xb.n_slabs, xb.d_chunk_start, xb.d_band_clo, xb.d_word,   \
                       xb.d_table, xb.table_size, x, y, xb.d_partials, xb.d_tickets, alpha, beta,  \
                       xcd_map)
#ifdef SM_DEV
    // Development builds: ablations (SM_BAND2_ABLATE, results wrong) and the wave
    // priority (SM_BAND2_PRIO) of DESIGN.md §3.4b's measurements.
    static const int abl = [] {
        const char *e = dev_env("SM_BAND2_ABLATE");
        return e ? atoi(e) : 0;
    }();
    static const int prio = [] {
        const char *e = dev_env("SM_BAND2_PRIO");
        return e ? atoi(e) : 2;
    }();
    if (half2) {
        switch (abl) {
        case 0: SM_B2(0, 2, true, 3); break;
        case 8: SM_B2(8, 2, true, 3); break;
        case 2048: SM_B2(2048, 2, true, 3); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (dma3t) {
        if (abl != 0) return hipErrorInvalidValue;
        SM_B2(0, 2, true, 5);
        return hipGetLastError();
    }
    if (dmaw4 && abl != 2048) {
        if (abl == 0) SM_B2(0, 2, true, 9);
        else if (abl == 4096) {
            unsigned long long h[8] = {};
            void *sym = nullptr;
            if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_b2_prof)) != hipSuccess) return hipErrorInvalidValue;
            (void)hipMemsetAsync(sym, 0, sizeof(h), s);
            SM_B2(4096, 2, true, 9);
            (void)hipMemcpyAsync(h, sym, sizeof(h), hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
            const double wa = (double)(h[7] & 0xFFFFFFFFull), wl = (double)(h[7] >> 32);
            const double bands = (double)h[6] / (wa + wl);
            fprintf(stderr, "dmaw4 prof (cycles per band per wave; %.0f applying + %.0f loader waves, %.1f bands): "
                    "apply waves: entry wait %.0f apply %.0f barrier %.0f | loaders: issue %.0f dma wait %.0f "
                    "barrier %.0f\n", wa, wl, bands, h[0] / wa / bands, h[1] / wa / bands, h[2] / wa / bands,
                    h[3] / wl / bands, h[4] / wl / bands, h[5] / wl / bands);
        } else return hipErrorInvalidValue;
        return hipGetLastError();
    }
    if (dmaw && abl != 2048) {
        switch (abl) {
        case 4096: {
            unsigned long long h[8] = {};
            void *sym = nullptr;
            if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_b2_prof)) != hipSuccess) return hipErrorInvalidValue;
            (void)hipMemsetAsync(sym, 0, sizeof(h), s);
            SM_B2(4096, 2, true, 8);
            (void)hipMemcpyAsync(h, sym, sizeof(h), hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
            const double wa = (double)(h[7] & 0xFFFFFFFFull), wl = (double)(h[7] >> 32);
            const double bands = (double)h[6] / (wa + wl);
            fprintf(stderr, "dmaw prof (cycles per band per wave; %.0f applying + %.0f loader waves, %.1f bands): "
                    "apply waves: entry wait %.0f apply %.0f barrier %.0f | loaders: issue %.0f dma wait %.0f "
                    "barrier %.0f\n", wa, wl, bands, h[0] / wa / bands, h[1] / wa / bands, h[2] / wa / bands,
                    h[3] / wl / bands, h[4] / wl / bands, h[5] / wl / bands);
            break;
        }
        case 0: SM_B2(0, 2, true, 8); break;
        case 1: SM_B2(1, 2, true, 8); break;
        case 8: SM_B2(8, 2, true, 8); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (dma3tall && abl != 2048) {
        switch (abl) {
        case 0: SM_B2(0, 2, true, 6); break;
        case 1: SM_B2(1, 2, true, 6); break;
        case 8: SM_B2(8, 2, true, 6); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (dma3 && !cb) {
        if (abl != 0) return hipErrorInvalidValue;
        SM_B2(0, 2, false, 4);
        return hipGetLastError();
    }
    if (dma3 && abl != 2048) {
        switch (abl) {
        case 4096: {
            unsigned long long h[8] = {};
            void *sym = nullptr;
            if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_b2_prof)) != hipSuccess) return hipErrorInvalidValue;
            (void)hipMemsetAsync(sym, 0, sizeof(h), s);
            SM_B2(4096, 2, true, 4);
            (void)hipMemcpyAsync(h, sym, sizeof(h), hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
            const double wa = (double)(h[7] & 0xFFFFFFFFull), wl = (double)(h[7] >> 32);
            const double bands = (double)h[6] / (wa + wl);
            fprintf(stderr, "dma3 prof (cycles per band per wave; %.0f applying + %.0f loader waves, %.1f bands): "
                    "apply waves: entry wait %.0f apply %.0f barrier %.0f | loader: issue %.0f dma wait %.0f "
                    "barrier %.0f\n", wa, wl, bands, h[0] / wa / bands, h[1] / wa / bands, h[2] / wa / bands,
                    h[3] / wl / bands, h[4] / wl / bands, h[5] / wl / bands);
            break;
        }
        case 0:
            if (prio == 1) SM_B2(0, 1, true, 4);
            else if (prio == 3) SM_B2(0, 3, true, 4);
            else if (prio == 0) SM_B2(0, 0, true, 4);
            else SM_B2(0, 2, true, 4);
            break;
        case 1: SM_B2(1, 2, true, 4); break;
        case 8: SM_B2(8, 2, true, 4); break;
        case 512: SM_B2(512, 2, true, 4); break;
        case 520: SM_B2(520, 2, true, 4); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (wide3) {
        switch (abl) {
        case 0: SM_B2(0, 2, true, 2); break;
        case 4: SM_B2(4, 2, true, 2); break;
        case 8: SM_B2(8, 2, true, 2); break;
        case 32: SM_B2(32, 2, true, 2); break;
        case 2048: SM_B2(2048, 2, true, 2); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (tall) {
        if (abl == 8) {
            if (cb) SM_B2(8, 2, true, 1); else SM_B2(8, 2, false, 1);
            return hipGetLastError();
        }
        if (abl != 0) return hipErrorInvalidValue;
        if (cb) SM_B2(0, 2, true, 1); else SM_B2(0, 2, false, 1);
        return hipGetLastError();
    }
    if (cb) {
        switch (abl) {
        case 0:
            if (prio == 0) SM_B2(0, 0, true, 0);
            else if (prio == 1) SM_B2(0, 1, true, 0);
            else if (prio == 3) SM_B2(0, 3, true, 0);
            else SM_B2(0, 2, true, 0);
            break;
        case 1: SM_B2(1, 2, true, 0); break;
        case 2: SM_B2(2, 2, true, 0); break;
        case 4: SM_B2(4, 2, true, 0); break;
        case 8: SM_B2(8, 2, true, 0); break;
        case 32: SM_B2(32, 2, true, 0); break;
        case 64: SM_B2(64, 2, true, 0); break;
        case 128: SM_B2(128, 2, true, 0); break;
        case 256: SM_B2(256, 2, true, 0); break;
        case 512: SM_B2(512, 2, true, 0); break;
        case 516: SM_B2(516, 2, true, 0); break;
        case 513: SM_B2(513, 2, true, 0); break;
        case 1024: {
            unsigned long long h[8] = {};
            void *sym = nullptr;
            if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_b2_prof)) != hipSuccess) return hipErrorInvalidValue;
            (void)hipMemsetAsync(sym, 0, sizeof(h), s);
            SM_B2(1024, 2, true, 0);
            (void)hipMemcpyAsync(h, sym, sizeof(h), hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
            const double w = (double)h[7], bands = (double)h[6] / w;
            fprintf(stderr, "cband prof (cycles per wave; %.0f waves, %.1f bands): prologue %.0f | per band: "
                    "x store %.0f apply %.0f e-load %.0f barrier %.0f | epilogue %.0f\n", w, bands,
                    h[0] / w, h[1] / w / bands, h[2] / w / bands, h[3] / w / bands, h[4] / w / bands, h[5] / w);
            break;
        }
        case 2048: {
            const int nt = (int)std::min<int64_t>(grid.x, 4096);
            std::vector<unsigned long long> h((size_t)3 * nt);
            void *sym = nullptr;
            if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_b2_ts)) != hipSuccess) return hipErrorInvalidValue;
            if (dma3) SM_B2(2048, 2, true, 4);
            else if (dmaw) SM_B2(2048, 2, true, 8);
            else if (dmaw4) SM_B2(2048, 2, true, 9);
            else if (dma3tall) SM_B2(2048, 2, true, 6);
            else SM_B2(2048, 2, true, 0);
            (void)hipMemcpyAsync(h.data(), sym, h.size() * 8, hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
            unsigned long long t0 = ~0ull;
            for (int i = 0; i < nt; i++) t0 = std::min(t0, h[3 * i]);
            std::vector<double> st(nt), lp(nt), ep(nt), en(nt);
            for (int i = 0; i < nt; i++) {
                st[i] = (h[3 * i] - t0) * 0.01;                 // us (100 MHz)
                lp[i] = (h[3 * i + 1] - h[3 * i]) * 0.01;
                ep[i] = (h[3 * i + 2] - h[3 * i + 1]) * 0.01;
                en[i] = (h[3 * i + 2] - t0) * 0.01;
            }
            auto pr = [](const char *nm, std::vector<double> v) {
                std::sort(v.begin(), v.end());
                const size_t k = v.size();
                fprintf(stderr, "  %-9s min %6.2f p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us\n", nm, v[0],
                        v[k / 10], v[k / 2], v[9 * k / 10], v[k - 1]);
            };
            fprintf(stderr, "cband tile timeline (%d tiles):\n", nt);
            pr("start", st);
            pr("loop", lp);
            pr("epilogue", ep);
            pr("end", en);
            if (dev_env("SM_B2_TS_DUMP")) {
                for (int i = 0; i < nt; i++)
                    fprintf(stderr, "  tile %4d start %6.2f loop %6.2f epi %6.2f\n", i, st[i], lp[i], ep[i]);
            }
            break;
        }
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    switch (abl) {
    case 0:
        if (prio == 0) SM_B2(0, 0, false, 0); else SM_B2(0, 2, false, 0);
        break;
    case 1: SM_B2(1, 2, false, 0); break;
    case 2: SM_B2(2, 2, false, 0); break;
    case 4: SM_B2(4, 2, false, 0); break;
    case 8: SM_B2(8, 2, false, 0); break;
    case 16: SM_B2(16, 2, false, 0); break;
    default: return hipErrorInvalidValue;
    }
#else
    if (wide3) return hipErrorInvalidValue;   // development builds only
    if (half2) {
        SM_B2(0, 2, true, 3);
    } else if (dma3) {
        if (cb) SM_B2(0, 2, true, 4); else SM_B2(0, 2, false, 4);
    } else if (dma3t) {
        SM_B2(0, 2, true, 5);
    } else if (dma3tall) {
        SM_B2(0, 2, true, 6);
    } else if (dmaw) {
        SM_B2(0, 2, true, 8);
    } else if (dmaw4) {
        SM_B2(0, 2, true, 9);
    } else if (tall) {
        if (cb) SM_B2(0, 2, true, 1); else SM_B2(0, 2, false, 1);
    } else {
        if (cb) SM_B2(0, 2, true, 0); else SM_B2(0, 2, false, 0);
    }
#endif
#undef SM_B2
    return hipGetLastError();
}

}  // namespace smamd
