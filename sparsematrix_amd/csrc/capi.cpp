// capi.cpp -- the extern "C" boundary of libsparsematrix_amd.so
// (include/sparsematrix.h).  Host-side C++: argument checks, device memory,
// uploads, planning and kernel dispatch.  All arithmetic runs in the HIP
// kernels of kernels.hip; there is no CPU compute path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <limits>
#include <memory>
#include <string>
#include <vector>

#include "ccsell.h"
#include "sweep.h"
#include "encode.h"
#include "gcb.h"
#include "sm_internal.h"
#include "sell.h"
#include "xband.h"

using namespace smamd;

namespace {

thread_local std::string g_err;

sm_status fail(sm_status s, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return s;
}

sm_status hip_fail(hipError_t e, const char *what) {
    return fail(e == hipErrorOutOfMemory ? SM_ERR_OUT_OF_MEMORY : SM_ERR_HIP, "%s: %s (%d)", what,
                hipGetErrorString(e), (int)e);
}

#define SM_TRY_HIP(call)                                    \
    do {                                                    \
        hipError_t e_ = (call);                             \
        if (e_ != hipSuccess) return hip_fail(e_, #call);   \
    } while (0)

constexpr int64_t kI32Max = std::numeric_limits<int32_t>::max();

// Makes `dev` current for the scope and restores the caller's device.
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) err = hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

template <typename T>
hipError_t dev_alloc(T **p, int64_t count, int64_t &acct) {
    const size_t bytes = (size_t)std::max<int64_t>(count, 1) * sizeof(T);
    hipError_t e = hipMalloc((void **)p, bytes);
    if (e == hipSuccess) acct += (int64_t)bytes;
    return e;
}

void free_xband_dev(XbandDev &h) {
    (void)hipFree(h.d_chunk_start);
    (void)hipFree(h.d_word);
    (void)hipFree(h.d_val);
    (void)hipFree(h.d_partials);
    (void)hipFree(h.d_tickets);
    (void)hipFree(h.d_band_clo);
    (void)hipFree(h.d_table);
    (void)hipFree(h.d_pace);
    h = XbandDev();
}

// The native-format plan (upload_native); left empty, as a matrix without one.
void free_native_dev(NativeDev &n) {
    for (void *p : {(void *)n.d_pos, (void *)n.d_val, (void *)n.d_beg, (void *)n.d_end, (void *)n.d_col,
                    (void *)n.d_table, (void *)n.d_pbatch, (void *)n.d_bmeta, (void *)n.d_boff,
                    (void *)n.d_lists, (void *)n.d_hdr})
        (void)hipFree(p);
    n = NativeDev{};
}

void free_device(sm_matrix *m) {
    DeviceGuard g(m->device);
    (void)hipFree(m->d_row_ptr);
    (void)hipFree(m->d_col);
    (void)hipFree(m->d_val);
    (void)hipFree(m->plan.d_tiles);
    (void)hipFree(m->plan.d_merge);
    (void)hipFree(m->plan.d_merge_corner);
    (void)hipFree(m->plan.d_mstage_w);
    (void)hipFree(m->plan.d_mstage_z);
    (void)hipFree(m->plan.d_mstage_tab);
    (void)hipFree(m->plan.d_long_rows);
    (void)hipFree(m->plan.d_long_ptr);
    (void)hipFree(m->plan.d_chunks);
    (void)hipFree(m->plan.d_partials);
    free_xband_dev(m->plan.xb);
    (void)hipFree(m->plan.d_perm);
    (void)hipFree(m->plan.d_rcol);
    (void)hipFree(m->plan.d_xperm);
    for (SellDev *d : {&m->plan.sell, &m->plan.xsell})
        for (void *p : {(void *)d->d_off, (void *)d->d_len, (void *)d->d_row, (void *)d->d_row_len,
                        (void *)d->d_col, (void *)d->d_val, (void *)d->d_table, (void *)d->d_long_rows,
                        (void *)d->d_long_ptr, (void *)d->d_partials})
            (void)hipFree(p);
    (void)hipFree(m->plan.cc.d_off);
    (void)hipFree(m->plan.cc.d_len);
    (void)hipFree(m->plan.cc.d_row);
    (void)hipFree(m->plan.cc.d_row_len);
    (void)hipFree(m->plan.cc.d_word);
    (void)hipFree(m->plan.cc.d_val);
    (void)hipFree(m->plan.cc.d_table);
    free_native_dev(m->plan.nat);
    (void)hipFree(m->plan.sw.d_block_chunk);
    (void)hipFree(m->plan.sw.d_ent);
    (void)hipFree(m->plan.sw.d_table);
    free_xband_dev(m->plan.hot);
    (void)hipFree(m->d_ws);
    if (m->ws_ready) (void)hipEventDestroy(m->ws_ready);
    if (m->scratch_ready) (void)hipEventDestroy(m->scratch_ready);
    m->scratch_ready = nullptr;
    m->scratch_recorded = false;
    m->d_ws = nullptr;
    m->ws_bytes = 0;
    m->ws_ready = nullptr;
    m->d_row_ptr = m->d_col = nullptr;
    m->d_val = nullptr;
    m->plan = Plan();
}

// SM_DEBUG_SYNC=1: synchronise after every launch and report the failing call
// (fault attribution; it changes no result, only the timing).
bool debug_sync() {
    static const bool on = [] {
        const char *e = getenv("SM_DEBUG_SYNC");
        return e && atoi(e) != 0;
    }();
    return on;
}

hipError_t after_launch(hipError_t e, hipStream_t s, const char *what) {
    if (e != hipSuccess || !debug_sync()) return e;
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) fprintf(stderr, "[sparsematrix_amd] %s failed: %s\n", what, hipGetErrorString(e));
    return e;
}

// Layout options: the caller's sm_build_opts with defaults for what it leaves out
// (struct_size) and, in -DSM_DEV builds only, the SM_* development variables on top.
BuildOpts resolve_opts(const sm_build_opts *o) {
    BuildOpts r;
    if (o) {
        sm_build_opts d;
        sm_build_opts_init(&d);
        const size_t n = std::min<size_t>(sizeof(d), (size_t)std::max<int32_t>(o->struct_size, 0));
        memcpy(&d, o, n);
        r.layout = d.layout;
        r.band_slabs = d.band_slabs;
        r.band_tall = d.band_tall;
        r.gather_band_log2 = d.gather_band_log2;
        r.sell = d.sell;
        r.sell_codebook = d.sell_codebook;
        r.sell_max_len = d.sell_max_len;
        r.sell_streams = d.sell_streams;
        r.sell_sigma = d.sell_sigma;
        r.relabel = d.relabel;
        r.tile_nnz = d.tile_nnz;
        r.ccsell = d.ccsell;
        r.ccsell_chunk_log2 = d.ccsell_chunk_log2;
        r.hot_cols = d.hot_cols;
        r.exact_sell = d.exact_sell;
        r.band_slab0_permille = d.band_slab0_permille;
        r.merge_stage = d.merge_stage;
        r.host_build = d.host_build;
    }
    if (const char *e = dev_env("SM_XBAND")) r.layout = atoi(e) ? SM_LAYOUT_BANDS : SM_LAYOUT_NO_BANDS;
    if (const char *e = dev_env("SM_XBAND_KIND")) {
        static const char *names[] = {"", "exact", "blocked", "gather", "band2", "cband"};
        for (int k = 1; k <= 5; ++k)
            if (strcmp(e, names[k]) == 0) r.layout = k;
        if (strcmp(e, "sweep") == 0) r.layout = SM_LAYOUT_SWEEP;
        if (strcmp(e, "gcb") == 0) r.layout = SM_LAYOUT_GCB;
    }
    if (const char *e = dev_env("SM_BAND_TALL")) r.band_tall = atoi(e);
    if (const char *e = dev_env("SM_BAND2_SLABS")) r.band_slabs = atoi(e);
    if (const char *e = dev_env("SM_BAND_SLAB0")) r.band_slab0_permille = atoi(e);
    if (const char *e = dev_env("SM_XBAND_GBAND")) r.gather_band_log2 = atoi(e);
    if (const char *e = dev_env("SM_RELABEL")) r.relabel = atoi(e);
    if (const char *e = dev_env("SM_SELL")) r.sell = atoi(e) ? -1 : 0;
    if (const char *e = dev_env("SM_SELL_CB")) r.sell_codebook = atoi(e) ? -1 : 0;
    if (const char *e = dev_env("SM_SELL_MAX")) r.sell_max_len = atoi(e);
    if (const char *e = dev_env("SM_SELL_SIGMA")) r.sell_sigma = atoll(e);
    if (const char *e = dev_env("SM_SELL_STREAMS")) r.sell_streams = atoi(e);
    if (const char *e = dev_env("SM_TILE_NNZ")) r.tile_nnz = atoi(e);
    if (const char *e = dev_env("SM_CCSELL")) r.ccsell = atoi(e);
    if (const char *e = dev_env("SM_CCSELL_CHUNK")) r.ccsell_chunk_log2 = atoi(e);
    if (const char *e = dev_env("SM_HOT_COLS")) r.hot_cols = atoi(e);
    if (const char *e = dev_env("SM_MERGE_STAGE")) r.merge_stage = atoi(e);
    if (const char *e = dev_env("SM_HOST_BUILD")) r.host_build = atoi(e);
    return r;
}

sm_status check_opts(const sm_build_opts *o) {
    if (!o) return SM_OK;
    if (o->struct_size < (int32_t)(2 * sizeof(int32_t)))
        return fail(SM_ERR_INVALID_ARG, "sm_build_opts.struct_size %d: call sm_build_opts_init",
                    o->struct_size);
    const BuildOpts r = resolve_opts(o);
    if (r.layout < SM_LAYOUT_AUTO || r.layout > SM_LAYOUT_GCB)
        return fail(SM_ERR_INVALID_ARG, "unknown layout %d", r.layout);
    if (r.band_slabs < 0 || r.band_slabs > 16) return fail(SM_ERR_INVALID_ARG, "band_slabs not in [0, 16]");
    if (r.band_tall != 0 && r.band_tall != 4 && r.band_tall != 6)
        return fail(SM_ERR_INVALID_ARG, "band_tall must be 0 (dma3), 4 (dma3) or 6 (wide)");
    if (r.gather_band_log2 != 0 && (r.gather_band_log2 < 13 || r.gather_band_log2 > 15))
        return fail(SM_ERR_INVALID_ARG, "gather_band_log2 must be 0 or 13..15");
    if (r.tile_nnz != 0 && r.tile_nnz != 1024 && r.tile_nnz != 2048 && r.tile_nnz != 4096 &&
        r.tile_nnz != 8192)
        return fail(SM_ERR_INVALID_ARG, "tile_nnz must be 0, 1024, 2048, 4096 or 8192");
    if (r.sell_max_len < 0 || r.sell_streams < 0 || r.sell_sigma < 0)
        return fail(SM_ERR_INVALID_ARG, "negative sell option");
    if (r.ccsell_chunk_log2 != 0 && (r.ccsell_chunk_log2 < 8 || r.ccsell_chunk_log2 > 24))
        return fail(SM_ERR_INVALID_ARG, "ccsell_chunk_log2 must be 0 or 8..24");
    if (r.hot_cols < -1) return fail(SM_ERR_INVALID_ARG, "hot_cols must be -1, 0 or positive");
    if (r.exact_sell < -1 || r.exact_sell > 1) return fail(SM_ERR_INVALID_ARG, "exact_sell must be -1, 0 or 1");
    if (r.band_slab0_permille != 0 && (r.band_slab0_permille < 500 || r.band_slab0_permille > 1000))
        return fail(SM_ERR_INVALID_ARG, "band_slab0_permille must be 0 or 500..1000");
    if (r.merge_stage != 0 && r.merge_stage != 1) return fail(SM_ERR_INVALID_ARG, "merge_stage must be 0 or 1");
    if (r.host_build != 0 && r.host_build != 1) return fail(SM_ERR_INVALID_ARG, "host_build must be 0 or 1");
    return SM_OK;
}

int32_t tile_nnz_setting(const sm_matrix *m) {
    const int v = m->opts.tile_nnz;
    return (v == 1024 || v == 2048 || v == 4096 || v == 8192) ? v : kTileNnz;
}

bool kind_forced(const sm_matrix *m) {
    return (m->opts.layout >= SM_LAYOUT_EXACT && m->opts.layout <= SM_LAYOUT_CBAND) ||
           m->opts.layout == SM_LAYOUT_GCB;
}

// Column-band layout.  SM_LAYOUT_NO_BANDS disables it,
// SM_LAYOUT_BANDS (or a forced kind) builds it; otherwise it is built when sweeping x
// through every tile's LDS costs less than the random gathers it replaces.  Cost model
// from profiles/r01_microbench.txt: a tile streams x into LDS at ~85 GB/s per CU
// (~22 TB/s chip-wide) while 4-byte gathers run at 75-200 G/s by the size of x,
// so the sweep wins while its bytes stay under ~20x the matrix's 8 B per term.
// AUTO's kind: cband (balanced bands of codebook words, kernels_band2.hip; band2 when
// the values take more than 255 bit patterns; it falls back to blocked when its bands
// would be < 70 % filled), or gather for wide matrices -- measured per rank of the
// bench's row partition (1M rows, 16 terms per row), blocked vs gather
// with 16K- / 32K-column bands: 1M columns 46 vs 59 / -, 2M 59 vs 60 / 66, 4M 85 vs
// 77 / 73, 8M 145 vs - / 93 us.  Past ~3M columns each blocked tile sweeps more x
// through LDS than gathering its terms' x costs.
constexpr int64_t kGatherCols = 3 * ((int64_t)1 << 20);   // gather kind: > 3M columns
// Gathered chunk bands (gcb.h): past 16M columns (config 5's 64M-column rank slices: 0.83 vs
// 1.61 ms for the gather kind) -- the gather kind's 32K-column bands hold too
// few terms there; where the gather kind's own cost model accepts a band layout.
constexpr int64_t kGcbCols = (int64_t)1 << 24;

XbKind xband_kind_setting(const sm_matrix *m) {
    switch (m->opts.layout) {
    case SM_LAYOUT_EXACT: return kXbExact;
    case SM_LAYOUT_BLOCKED: return kXbBlocked;
    case SM_LAYOUT_GATHER: return kXbGather;
    case SM_LAYOUT_BAND2: return kXbBand2;
    case SM_LAYOUT_CBAND: return kXbCband;
    case SM_LAYOUT_GCB: return kXbGcb;
    default: break;
    }
    return m->n_cols >= kGcbCols ? kXbGcb : m->n_cols > kGatherCols ? kXbGather : kXbCband;
}

// Sweeping x through LDS (or walking its bands) pays when the L2 -> LDS bytes of
// one kind's row blocks stay within 20x the matrix stream.  The gather kind sweeps no
// x: its cost is its bands' skeleton plus its terms, set against the sliced ELL's cost
// per term on wide uniform matrices -- constants from the two measured wide shapes
// (config 2 rows at 8M columns: 16K bands of 1K terms, 93 us; config 5's rank slice,
// 8M x 64M: 1M bands of 128 terms, 1.60 ms; its ccsell 2.30 ms = 17 ps per term).
static bool gather_cost_ok(const sm_matrix *m) {
    // Calibrated on uniform rows: skewed ones (longest row > 64x the mean, e.g. R-MAT)
    // keep the sliced ELL, whose long-row segments balance them.
    if ((double)m->plan.max_row_nnz > 64.0 * (double)m->nnz / (double)std::max<int64_t>(1, m->n_rows))
        return false;
    const int64_t nblk = (m->n_rows + (1 << kXbGatherRowsLog2) - 1) >> kXbGatherRowsLog2;
    const double bands = (double)nblk * (double)((m->n_cols + (1 << kXbGatherWideBandLog2) - 1) >>
                                                 kXbGatherWideBandLog2);
    const double per_band_us = 0.25 + 1.2e-3 * (double)m->nnz / bands;
    const double gather_us = bands / 256.0 * per_band_us;
    const double sell_us = 1.7e-5 * (double)m->nnz;
    return gather_us < sell_us;
}

// Below this many terms AUTO keeps the sorted sliced ELL instead of a swept band layout: a
// band SpMV carries ~20 us of fixed cost (x staging per tile, the slab hand-off) that small
// matrices do not amortise, and their few row blocks leave CUs idle (16K rows: 16 tiles).
// Uniform 16-per-row squares, eager SpMV incl. launch (tools/small_auto_ab.py,
// profiles/r06_small_auto_ab.txt): 2^18 rows (4.2 M terms) cband 31.3 vs sell 22.3 us,
// 2^19 (8.4 M) 34.6 vs 41.6 us.
constexpr int64_t kBandMinNnz = 6 * ((int64_t)1 << 20);

static bool xband_cost_ok(const sm_matrix *m, XbKind kind) {
    if ((kind == kXbGather || kind == kXbGcb) && m->n_cols > kGatherCols && m->opts.gather_band_log2 == 0)
        return gather_cost_ok(m);   // gcb: ~2x faster than the gather kind it is priced as
    if (m->nnz < kBandMinNnz) return false;
    const int rows_log2 = kind == kXbExact    ? kXbExactRowsLog2
                          : kind == kXbBand2 || kind == kXbCband ? kB2RowBits
                          : kind == kXbGather ? kXbGatherRowsLog2
                                              : kXbBlockedRowsLog2;
    const int64_t nblk = (m->n_rows + (1 << rows_log2) - 1) >> rows_log2;
    const double x_sweep = (double)nblk * 4.0 * (double)m->n_cols;   // L2 -> LDS bytes
    const double stream = 8.0 * (double)m->nnz;                      // HBM bytes
    return x_sweep <= 20.0 * stream && m->n_cols >= 8192;
}

bool want_xband(const sm_matrix *m) {
    const int32_t L = m->opts.layout;
    if (L == SM_LAYOUT_NO_BANDS || L == SM_LAYOUT_SWEEP) return false;
    if (m->nnz == 0 || m->n_rows == 0) return false;
    if (L != SM_LAYOUT_AUTO) return true;   // a forced kind, or SM_LAYOUT_BANDS
    return xband_cost_ok(m, xband_kind_setting(m));
}

// Balanced-band layout (band2.cpp, kernels_band2.hip): slabs so there are about
// kXbTargetTiles tiles of <= 16K rows.  kind cband: 4-byte codebook words when the
// values take <= 255 distinct bit patterns, else (or kind band2) 8-byte entries.
// Builds into `d` the balanced bands of an n_rows x n_cols CSR (the matrix's own, or
// the hot column prefix of a relabeled graph); `forced`: keep mostly-padding bands.
// Geometry (sm_build_opts.band_tall): 0 = the default (dma3, both encodings: a loader wave
// stages x -- config 2 34.0-34.6 vs 36.9-37.1 us for the wide geometry with codebook words,
// 37.9-38.0 vs 38.6-38.7 with 8-byte entries), 4 = dma3, 6 = wide.  dma3
// bands that would be < 70 % full fall back to wide.
static sm_status build_band2(sm_matrix *m, XbandDev &d, int64_t n_rows, int64_t n_cols, int64_t nnz,
                             const int32_t *rp, const int32_t *col, const float *val, XbKind kind,
                             int32_t geo_opt, int32_t slabs, bool forced, int32_t slab0_permille = 1000) {
    const bool dma3 = geo_opt != 6;
    const B2Geom geom = dma3 ? (kind == kXbCband ? kB2Dma3Cb : kB2Dma3B2) : kB2Wide;
    const int64_t br = std::min<int64_t>(geom.block_rows, n_rows);
    const int64_t nblk = (n_rows + br - 1) / br;
    int32_t want = (int32_t)std::max<int64_t>(
        1, std::min<int64_t>(16, (kXbTargetTiles + nblk - 1) / nblk));
    if (slabs > 0) want = std::max(1, std::min(16, slabs));
    std::vector<float> table;
    std::vector<uint8_t> ids;
    const bool cb = kind == kXbCband && codebook_ids(val, nnz, table, ids);
    Band2Host bh;
    B2Geom g = dma3 ? (cb ? kB2Dma3Cb : kB2Dma3B2) : kB2Wide;
    // Bands are fixed slots of g.chunks() * 64 entries: where a slab's density leaves
    // them mostly dummies (wide or very sparse matrices), the padding would cost more HBM
    // bytes than the layout saves -- decline unless forced (SM_LAYOUT_BAND2 / CBAND).
    auto fits = [&](const B2Geom &gg) {
        if (!band2_build(rp, col, val, n_rows, n_cols, want, bh, cb ? ids.data() : nullptr, gg, slab0_permille))
            return false;
        return forced || bh.n_bands == 0 ||
               (double)bh.real_terms >= 0.7 * (double)bh.n_bands * gg.chunks() * 64;
    };
    bool ok = fits(g);
    if (!ok && g.nch != 0) {   // dma3 did not fit: wide
        g = kB2Wide;
        ok = fits(g);
    }
    if (!ok) return SM_OK;
    std::vector<uint8_t>().swap(ids);
    const int64_t band_words = (int64_t)(cb ? 64 : 128) * g.chunks();
    const int64_t ntile = (int64_t)bh.n_blocks * bh.n_slabs;
    SM_TRY_HIP(dev_alloc(&d.d_chunk_start, ntile + 1, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_band_clo, std::max<int64_t>(1, bh.n_bands), m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_word, std::max<int64_t>(1, bh.n_bands * band_words), m->device_bytes));
    if (cb) {
        SM_TRY_HIP(dev_alloc(&d.d_table, 256, m->device_bytes));
        SM_TRY_HIP(hipMemset(d.d_table, 0, 256 * sizeof(float)));
        if (!table.empty())
            SM_TRY_HIP(hipMemcpy(d.d_table, table.data(), table.size() * 4, hipMemcpyHostToDevice));
        d.table_size = (int32_t)table.size();
    }
    if (bh.n_slabs > 1) {
        const int64_t ps = (n_rows + 3) & ~(int64_t)3;   // 16-byte aligned partial rows
        // One partial per slab: the beta-last hand-off (kernels_band2.hip SM_B2_BL) publishes
        // slab 0's sums too (the other form writes them into y and leaves the last one unused).
        SM_TRY_HIP(dev_alloc(&d.d_partials, (int64_t)bh.n_slabs * ps, m->device_bytes));
        SM_TRY_HIP(dev_alloc(&d.d_tickets, 4 * (int64_t)bh.n_blocks, m->device_bytes));
        SM_TRY_HIP(hipMemset(d.d_tickets, 0, (size_t)bh.n_blocks * 4 * sizeof(int32_t)));
    }
    SM_TRY_HIP(hipMemcpy(d.d_chunk_start, bh.tile_band_start.data(), (size_t)(ntile + 1) * 4,
                         hipMemcpyHostToDevice));
    if (bh.n_bands > 0) {
        SM_TRY_HIP(hipMemcpy(d.d_band_clo, bh.band_clo.data(), (size_t)bh.n_bands * 4,
                             hipMemcpyHostToDevice));
        SM_TRY_HIP(hipMemcpy(d.d_word, bh.ent.data(), (size_t)(bh.n_bands * band_words) * 4,
                             hipMemcpyHostToDevice));
    }
    d.kind = cb ? kXbCband : kXbBand2;
    d.threads = 1024;
    d.block_rows = bh.block_rows;
    d.band_cols = g.window;
    d.n_bands = (int32_t)std::min<int64_t>(bh.n_bands, INT32_MAX);
    d.n_slabs = bh.n_slabs;
    d.slab_bands = bh.slab_cols;
    d.slab0_cols = bh.slab0_cols;
    d.n_chunks = bh.n_bands * g.chunks();
    d.max_chunks_per_band = bh.max_bands_per_tile;
    d.n_blocks = bh.n_blocks;
    return SM_OK;
}

static sm_status upload_band2(sm_matrix *m, const int32_t *rp, const int32_t *col,
                              const float *val, XbKind kind) {
    // Geometry: band_tall (xband.h B2Geom, build_band2).
    // Slab 0's tile loads and scales y (64 KiB per 16K-row block from HBM) before its first
    // band: on config 2 its band loop ended 1.5-2.3 us after the other slabs' (per-tile
    // timeline, profiles/r05_dma3_tile_timeline_dump.txt).  Narrower slab-0 tiles did not
    // shorten the kernel (kB2Slab0Permille), so AUTO keeps even slabs; the option stays.
    const int32_t p0 = m->opts.band_slab0_permille > 0 ? m->opts.band_slab0_permille : kB2Slab0Permille;
    return build_band2(m, m->plan.xb, m->n_rows, m->n_cols, m->nnz, rp, col, val, kind,
                       m->opts.band_tall, m->opts.band_slabs, kind_forced(m), p0);
}

// Gathered chunk bands (gcb.h, kernels_gcb.hip): 32K-row tiles where the rows make at
// least 256 of them (one per CU), else 16K-row tiles; slabs so the tiles reach 256.
static void gcb_geometry(const sm_matrix *m, int &rows_log2, int32_t &slabs) {
    rows_log2 = m->n_rows >= ((int64_t)kXbTargetTiles << 15) ? 15 : 14;
    const int64_t nblk = (m->n_rows + ((int64_t)1 << rows_log2) - 1) >> rows_log2;
    slabs = (int32_t)std::max<int64_t>(1, std::min<int64_t>(16, (kXbTargetTiles + nblk - 1) / nblk));
    if (m->opts.band_slabs > 0) slabs = m->opts.band_slabs;
}

// The rest of a built gcb layout (its bands already in d_chunk_start / d_band_clo / d_word):
// slab partials, hand-off and pacing words, the geometry.
static sm_status gcb_finish(sm_matrix *m, const GcbHost &gh) {
    XbandDev &d = m->plan.xb;
    if (gh.n_slabs > 1) {
        const int64_t ps = (m->n_rows + 3) & ~(int64_t)3;   // 16-byte aligned partial rows
        SM_TRY_HIP(dev_alloc(&d.d_partials, (int64_t)(gh.n_slabs - 1) * ps, m->device_bytes));
        SM_TRY_HIP(dev_alloc(&d.d_tickets, 4 * (int64_t)gh.n_blocks, m->device_bytes));
        SM_TRY_HIP(hipMemset(d.d_tickets, 0, (size_t)gh.n_blocks * 4 * sizeof(int32_t)));
    }
    // Column pacing (kernels_gcb.hip): per dispatch group, a started count and one arrival
    // count per 2^18-column checkpoint, monotonic across launches.
    d.pace_k = (int32_t)((m->n_cols + kGcbMaxWindow - 1) / kGcbMaxWindow);
    SM_TRY_HIP(dev_alloc(&d.d_pace, 8 * (1 + (int64_t)d.pace_k), m->device_bytes));
    SM_TRY_HIP(hipMemset(d.d_pace, 0, (size_t)8 * (1 + d.pace_k) * sizeof(int32_t)));
    d.kind = kXbGcb;
    d.threads = 1024;
    d.block_rows = gh.block_rows;
    d.band_cols = gh.window;
    d.n_bands = (int32_t)std::min<int64_t>(gh.n_bands, INT32_MAX);
    d.n_slabs = gh.n_slabs;
    d.slab_bands = gh.slab_cols;
    d.n_chunks = gh.n_bands * kGcbChunks;
    d.max_chunks_per_band = gh.max_bands_per_tile;
    d.n_blocks = gh.n_blocks;
    return SM_OK;
}

static sm_status upload_gcb(sm_matrix *m, const int32_t *rp, const int32_t *col, const float *val) {
    int rows_log2 = 0;
    int32_t slabs = 1;
    gcb_geometry(m, rows_log2, slabs);
    GcbHost gh;
    if (!gcb_build(rp, col, val, m->n_rows, m->n_cols, rows_log2, slabs, kGcbMaxWindow, gh)) return SM_OK;
    XbandDev &d = m->plan.xb;
    const int64_t ntile = (int64_t)gh.n_blocks * gh.n_slabs;
    SM_TRY_HIP(dev_alloc(&d.d_chunk_start, ntile + 1, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_band_clo, std::max<int64_t>(1, gh.n_bands), m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_word, std::max<int64_t>(1, gh.n_bands * kGcbBandWords), m->device_bytes));
    SM_TRY_HIP(hipMemcpy(d.d_chunk_start, gh.tile_band_start.data(), (size_t)(ntile + 1) * 4,
                         hipMemcpyHostToDevice));
    if (gh.n_bands > 0) {
        SM_TRY_HIP(hipMemcpy(d.d_band_clo, gh.band_clo.data(), (size_t)gh.n_bands * 4, hipMemcpyHostToDevice));
        SM_TRY_HIP(hipMemcpy(d.d_word, gh.ent.data(), (size_t)gh.n_bands * kGcbBandWords * 4,
                             hipMemcpyHostToDevice));
    }
    return gcb_finish(m, gh);
}

sm_status upload_xband(sm_matrix *m, const int32_t *rp, const int32_t *col, const float *val,
                       XbKind kind) {
    if (kind == kXbGcb) return upload_gcb(m, rp, col, val);
    if (kind == kXbBand2 || kind == kXbCband) {
        const sm_status st = upload_band2(m, rp, col, val, kind);
        if (st == SM_OK && m->plan.xb.n_blocks == 0 && !kind_forced(m))
            return upload_xband(m, rp, col, val, kXbBlocked);   // declined: blocked kind
        return st;
    }
    // Gather kind: AUTO takes it past kGatherCols (3M columns) with bands of 32K
    // columns -- fewer bands, hence fewer per-band barriers, for the same terms (8M
    // columns: 93 us with 32K bands vs 122 with 8K); the rank field shrinks to 3 bits,
    // ample at < 0.25 terms per row per band.  A forced gather kind on a narrower
    // matrix keeps 8K-column bands.  gather_band_log2 = 13|14|15 forces the band width
    // (16K: measured slower than the blocked kind at 2M).
    const int gb = m->opts.gather_band_log2;
    const int gband_log2 = gb == 15 ? kXbGatherWideBandLog2
                           : gb == 14 ? kXbGatherWideBandLog2 - 1
                           : gb == 13 ? kXbGatherBandLog2
                           : m->n_cols > kGatherCols ? kXbGatherWideBandLog2
                                                     : kXbGatherBandLog2;
    const XbBits bits = kind == kXbExact    ? xb_bits(kXbExactBandLog2, kXbExactRowsLog2)
                        : kind == kXbGather ? xb_bits(gband_log2, kXbGatherRowsLog2)
                                            : xb_bits(kXbBlockedBandLog2, kXbBlockedRowsLog2);
    const int threads = kXbThreads;
    const int64_t target_tiles = (int64_t)kXbTargetTiles * (kXbThreads / threads);   // fill the CUs
    XbandHost xh;
    // Register capacity from the waves that hold entries: 12 on the blocked kind
    // (4 loader waves stage x), all 16 on the exact and gather kinds.
    const int entry_waves = kind == kXbBlocked ? kXbComputeWaves : threads / 64;
    if (!xband_build(rp, col, val, m->n_rows, m->n_cols, bits, entry_waves, xh,
                     kind == kXbGather)) {
        // The gather kind's wide bands leave 3-4 rank bits: a matrix with longer row
        // segments may still fit the blocked layout (5 bits, 8K-column bands).
        // Only where the blocked kind's own sweep cost still pays (its row blocks
        // differ from the gather kind's); otherwise the stream kernel serves it.
        if (kind == kXbGather && !kind_forced(m) &&
            (xband_cost_ok(m, kXbBlocked) || m->opts.layout == SM_LAYOUT_BANDS))
            return upload_xband(m, rp, col, val, kXbBlocked);
        return SM_OK;   // layout not applicable: the stream kernel serves this matrix
    }
    XbandDev &d = m->plan.xb;
    // Blocked: split the bands in slabs so there are >= kXbTargetTiles tiles.
    int32_t n_slabs = 1;
    if (kind != kXbExact) {
        // At most 64 slabs: the hand-off counts arrivals in 8 bits (kernels_xband.hip).
        const int64_t want = std::min<int64_t>(64, (target_tiles + xh.n_blocks - 1) / xh.n_blocks);
        n_slabs = (int32_t)std::max<int64_t>(1, std::min<int64_t>(want, xh.n_bands));
    }
    // Slabs of whole groups of 8 bands (the kernel steps bands 4 or 8 at a time).
    int32_t slab_bands = (xh.n_bands + n_slabs - 1) / n_slabs;
    slab_bands = (slab_bands + 7) & ~7;
    n_slabs = (xh.n_bands + slab_bands - 1) / slab_bands;
    std::vector<int32_t> cs32(xh.chunk_start.size());
    for (size_t i = 0; i < cs32.size(); i++) cs32[i] = (int32_t)xh.chunk_start[i];
    SM_TRY_HIP(dev_alloc(&d.d_chunk_start, (int64_t)cs32.size(), m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_word, (int64_t)xh.word.size(), m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_val, (int64_t)xh.val.size(), m->device_bytes));
    if (n_slabs > 1) {
        const int64_t ps = (m->n_rows + 3) & ~(int64_t)3;   // 16-byte aligned partial rows
        SM_TRY_HIP(dev_alloc(&d.d_partials, (int64_t)(n_slabs - 1) * ps, m->device_bytes));
        // Slab hand-off control words (kernels_xband.hip: started, arrive, done, pad).
        SM_TRY_HIP(dev_alloc(&d.d_tickets, 4 * (int64_t)xh.n_blocks, m->device_bytes));
        SM_TRY_HIP(hipMemset(d.d_tickets, 0, (size_t)xh.n_blocks * 4 * sizeof(int32_t)));
    }
    SM_TRY_HIP(hipMemcpy(d.d_chunk_start, cs32.data(), cs32.size() * 4, hipMemcpyHostToDevice));
    if (!xh.word.empty()) {
        SM_TRY_HIP(hipMemcpy(d.d_word, xh.word.data(), xh.word.size() * 4, hipMemcpyHostToDevice));
        SM_TRY_HIP(hipMemcpy(d.d_val, xh.val.data(), xh.val.size() * 4, hipMemcpyHostToDevice));
    }
    d.kind = kind;
    d.threads = threads;
    d.block_rows = xh.block_rows;
    d.band_cols = xh.band_cols;
    d.n_bands = xh.n_bands;
    d.n_slabs = n_slabs;
    d.slab_bands = slab_bands;
    d.n_chunks = xh.n_chunks;
    d.max_chunks_per_band = xh.max_chunks_per_band;
    d.n_blocks = xh.n_blocks;
    return SM_OK;
}

// Column relabeling for the stream kernel.  relabel = 0 disables
// it, 1 forces it; otherwise it is built when x is larger than an XCD's
// L2 (>= 2^20 columns), no band layout serves the matrix, there are at least as many
// terms as columns (the per-SpMV permutation of x is then cheap next to the
// product), and the column degrees are skewed: the busiest 1/16 of the columns hold
// >= 40 % of the terms (power-law graphs: R-MAT scale 24 has 87 % there).
bool want_relabel_size(const sm_matrix *m) {
    if (m->opts.relabel == 0) return false;
    if (m->nnz == 0 || m->n_cols == 0) return false;
    if (m->opts.relabel == 1) return true;
    return m->n_cols >= (1 << 20) && m->nnz >= m->n_cols && m->plan.xb.n_blocks == 0;
}

sm_status upload_relabel(sm_matrix *m, const int32_t *col) {
    const int64_t nc = m->n_cols, nnz = m->nnz;
    std::vector<int32_t> deg((size_t)nc, 0);
    for (int64_t e = 0; e < nnz; e++) deg[(size_t)col[e]]++;
    // new -> old, by descending degree; ties keep the original order (counting sort).
    int32_t dmax = 0;
    for (int32_t d : deg) dmax = std::max(dmax, d);
    std::vector<int64_t> start((size_t)dmax + 2, 0);
    for (int32_t d : deg) start[(size_t)(dmax - d) + 1]++;
    for (size_t i = 1; i < start.size(); i++) start[i] += start[i - 1];
    std::vector<int32_t> perm((size_t)nc), rank((size_t)nc);
    for (int64_t c = 0; c < nc; c++) {
        const int64_t j = start[(size_t)(dmax - deg[(size_t)c])]++;
        perm[(size_t)j] = (int32_t)c;
        rank[(size_t)c] = (int32_t)j;
    }
    if (m->opts.relabel != 1) {
        int64_t hot = 0;
        for (int64_t j = 0; j < nc / 16; j++) hot += deg[(size_t)perm[(size_t)j]];
        if ((double)hot < 0.4 * (double)nnz) return SM_OK;   // not skewed: no gain
    }
    std::vector<int32_t> rcol((size_t)nnz);
    for (int64_t e = 0; e < nnz; e++) rcol[(size_t)e] = rank[(size_t)col[e]];
    Plan &p = m->plan;
    SM_TRY_HIP(dev_alloc(&p.d_perm, nc + 4, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&p.d_rcol, nnz + kPadElems, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&p.d_xperm, nc + 4, m->device_bytes));
    // The SpMV permutes x by scattering it (coalesced reads, stores that never stall):
    // the device keeps the original -> new map.
    SM_TRY_HIP(hipMemcpy(p.d_perm, rank.data(), (size_t)nc * 4, hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(p.d_rcol, rcol.data(), (size_t)nnz * 4, hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemset(p.d_rcol + nnz, 0, kPadElems * sizeof(int32_t)));
    p.n_relabel = nc;
    return SM_OK;
}

// The merge path's column-sorted staging stream (kernels_merge.hip MergeStage), over the
// columns the merge kernel gathers with (the relabeled ones when the plan has them).
bool want_merge_stage(const sm_matrix *m) {
    return m->nnz > 0 && m->n_rows > 0 && m->opts.merge_stage == 1;
}

sm_status upload_merge_stage(sm_matrix *m, const int32_t *rp, const int32_t *col, const float *val) {
    std::vector<int32_t> rcol;
    if (m->plan.n_relabel > 0) {   // the relabeled columns (the plan keeps them on the device)
        rcol.resize((size_t)m->nnz);
        SM_TRY_HIP(hipMemcpy(rcol.data(), m->plan.d_rcol, (size_t)m->nnz * 4, hipMemcpyDeviceToHost));
        col = rcol.data();
    }
    std::vector<uint32_t> w;
    std::vector<uint16_t> z;
    std::vector<float> table;
    if (!merge_stage_build(rp, col, val, m->n_rows, m->n_cols, m->nnz, w, z, table)) return SM_OK;
    Plan &p = m->plan;
    SM_TRY_HIP(dev_alloc(&p.d_mstage_w, m->nnz, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&p.d_mstage_z, m->nnz, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&p.d_mstage_tab, 256, m->device_bytes));
    SM_TRY_HIP(hipMemcpy(p.d_mstage_w, w.data(), w.size() * 4, hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(p.d_mstage_z, z.data(), z.size() * 2, hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(p.d_mstage_tab, table.data(), 256 * 4, hipMemcpyHostToDevice));
    return SM_OK;
}

// Sorted sliced-ELL (sell.h, kernels_sell.hip) for every matrix no band layout
// serves (SM_SELL=0 disables it): faster than the stream kernel on uniform rows
// (config-2 shape without bands 100 vs 109 us, 2^17 rows 14.5 vs 15.8 us) and on
// R-MAT (1.91 vs 2.30 ms), and every row up to kSellMaxLen terms is summed in the
// reference's order (the stream kernel: rows up to 64).
bool want_sell(const sm_matrix *m) {
    if (m->opts.sell == 0) return false;
    return m->nnz > 0 && m->n_rows > 0 && m->plan.xb.n_blocks == 0 && m->plan.cc.n_slices == 0 &&
           m->plan.sw.n_blocks == 0;
}

sm_status upload_sell(sm_matrix *m, const int32_t *rp, const int32_t *col, const float *val,
                      int64_t nnz = -1, bool cols_relabeled = false, SellDev *target = nullptr,
                      int32_t max_len_override = 0) {
    Plan &p = m->plan;
    if (nnz < 0) nnz = m->nnz;
    std::vector<int32_t> rcol;
    const int32_t *c = col;
    if (p.n_relabel > 0 && !cols_relabeled) {   // the layout stores relabeled columns (x is permuted per SpMV)
        rcol.resize((size_t)m->nnz);
        SM_TRY_HIP(hipMemcpy(rcol.data(), p.d_rcol, (size_t)m->nnz * 4, hipMemcpyDeviceToHost));
        c = rcol.data();
    }
    // Rows up to max_len terms go to the slices (one lane each, in stored order); the
    // longer ones as max_len-term segments.  sell_max_len overrides the cap.
    const int32_t max_len = max_len_override > 0       ? max_len_override
                            : m->opts.sell_max_len > 0 ? m->opts.sell_max_len
                                                       : kSellMaxLen;
    // sell_sigma: sort within windows of that many rows (0: one window),
    // sell_streams: XCD streams of windows (default 8 with windows).
    const int64_t sigma = std::max<int64_t>(0, m->opts.sell_sigma);
    const int streams = m->opts.sell_streams > 0 ? m->opts.sell_streams : sigma > 0 ? 8 : 1;
    // Codebook form (sell_codebook = 0 disables it): values of <= 255 distinct bit
    // patterns and columns < 2^24 -- one 4-byte word per slot instead of column + value.
    std::vector<float> table;
    std::vector<uint8_t> ids;
    const bool cb = m->opts.sell_codebook != 0 && m->n_cols <= ((int64_t)1 << kSellCbColBits) &&
                    codebook_ids(val, nnz, table, ids);
    if (!cb) std::vector<uint8_t>().swap(ids);
    SellHost sh;
    sell_build(rp, c, val, m->n_rows, max_len, sh, sigma, streams, cb ? ids.data() : nullptr);
    std::vector<int32_t>().swap(rcol);
    std::vector<uint8_t>().swap(ids);
    if (sh.n_slices == 0) return SM_OK;
    if (sh.padded >= ((int64_t)1 << 31) - kSellLanes * kSellUnroll) return SM_OK;
    SellDev &d = target ? *target : p.sell;
    d.max_len = max_len;
    d.n_long = (int32_t)sh.long_rows.size();
    const int32_t n_parts = sh.long_ptr.back();
    SM_TRY_HIP(dev_alloc(&d.d_long_rows, d.n_long, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_long_ptr, d.n_long + 1, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_partials, n_parts, m->device_bytes));
    if (d.n_long) {
        SM_TRY_HIP(hipMemcpy(d.d_long_rows, sh.long_rows.data(), sh.long_rows.size() * 4, hipMemcpyHostToDevice));
        SM_TRY_HIP(hipMemcpy(d.d_long_ptr, sh.long_ptr.data(), sh.long_ptr.size() * 4, hipMemcpyHostToDevice));
    }
    SM_TRY_HIP(dev_alloc(&d.d_off, sh.n_slices, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_len, sh.n_slices, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_row, sh.n_slices * kSellLanes, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_row_len, sh.n_slices * kSellLanes, m->device_bytes));
    // + a zeroed tail of 32 slots per lane: unrolls past kSellUnroll read up to it.
    const int64_t tail = 32 * kSellLanes;
    SM_TRY_HIP(dev_alloc(&d.d_col, sh.padded + tail, m->device_bytes));
    SM_TRY_HIP(hipMemset(d.d_col + sh.padded, 0, (size_t)tail * 4));
    if (cb) {
        SM_TRY_HIP(dev_alloc(&d.d_table, std::max<int64_t>((int64_t)table.size(), 1), m->device_bytes));
        if (!table.empty())
            SM_TRY_HIP(hipMemcpy(d.d_table, table.data(), table.size() * 4, hipMemcpyHostToDevice));
        d.table_size = (int32_t)table.size();
    } else {
        SM_TRY_HIP(dev_alloc(&d.d_val, sh.padded + tail, m->device_bytes));
        SM_TRY_HIP(hipMemset(d.d_val + sh.padded, 0, (size_t)tail * 4));
    }
    SM_TRY_HIP(hipMemcpy(d.d_off, sh.off.data(), sh.off.size() * 8, hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(d.d_len, sh.len.data(), sh.len.size() * 4, hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(d.d_row, sh.row.data(), sh.row.size() * 4, hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(d.d_row_len, sh.row_len.data(), sh.row_len.size() * 4, hipMemcpyHostToDevice));
    if (sh.padded) {
        SM_TRY_HIP(hipMemcpy(d.d_col, sh.col.data(), (size_t)sh.padded * 4, hipMemcpyHostToDevice));
        if (!cb) SM_TRY_HIP(hipMemcpy(d.d_val, sh.val.data(), (size_t)sh.padded * 4, hipMemcpyHostToDevice));
    }
    d.n_slices = sh.n_slices;
    return SM_OK;
}

// SM_ALGO_EXACT: the fastest launch built for `m` that adds every output's terms in the
// reference's order (kernel.cc:780-796, sparse-matrix.cc:164-190) -- what the reference's
// C++ surface runs (sblas_shim.cpp).  The band kernels need x 16-byte aligned (`x16`).
// kAlgoExactSell: the unsegmented sliced ELL built for this (upload_exact_sell).
constexpr int kAlgoExactSell = 100;

int exact_algo(const sm_matrix *m, bool x16) {
    const Plan &pl = m->plan;
    if (pl.sw.n_blocks > 0) return SM_ALGO_XBAND;                                  // column-swept blocks
    if (pl.xb.n_blocks > 0 && pl.xb.n_slabs == 1 && x16) return SM_ALGO_XBAND;    // one slab of bands
    if (pl.cc.n_slices > 0) return SM_ALGO_SELL;                                    // column-chunked ELL
    if (pl.sell.n_slices > 0 && pl.sell.n_long == 0 && pl.hot.n_blocks == 0) return SM_ALGO_SELL;
    if (pl.max_row_nnz <= SM_SERIAL_ROW_MAX) return SM_ALGO_STREAM;                // serial rows only
    if (pl.xsell.n_slices > 0) return kAlgoExactSell;
    return SM_ALGO_PARITY;
}

// The unsegmented sliced ELL for SM_ALGO_EXACT (sm_build_opts.exact_sell): by default for
// matrices made by the CopyForm constructors -- the reference's own path, whose C++
// surface promises its results bit for bit -- when nothing else built keeps the order.
bool want_exact_sell(const sm_matrix *m) {
    if (m->nnz == 0 || m->n_rows == 0 || m->opts.exact_sell < 0) return false;
    if (m->opts.exact_sell == 0 && !m->from_index) return false;
    return exact_algo(m, true) == SM_ALGO_PARITY;
}

sm_status upload_exact_sell(sm_matrix *m, const int32_t *rp, const int32_t *col, const float *val) {
    // Rows never cut: the slice cap is the longest row (a lane walks its whole row).
    const int32_t cap = std::max<int32_t>(m->plan.max_row_nnz, 1);
    return upload_sell(m, rp, col, val, -1, false, &m->plan.xsell, cap);
}

// Column-chunked sorted sliced-ELL (ccsell.h, kernels_ccsell.hip):
// AUTO builds it instead of the sliced ELL when x is far larger than an XCD's L2
// (>= 2^23 columns = 32 MiB, 8 L2s' worth) and no band layout or relabeling serves
// the matrix -- a row-ordered ELL would gather every term's x from the Infinity Cache
// or HBM.  It declines (and the sliced ELL serves) when one row has more than 2048
// terms inside one column chunk.  ccsell = 0 / 1 never / always tries it.
// Column-swept row blocks (sweep.h, kernels_sweep.hip): forced by SM_LAYOUT_SWEEP.
bool want_sweep(const sm_matrix *m) {
    if (m->nnz == 0 || m->n_rows == 0 || m->plan.xb.n_blocks > 0) return false;
    if (m->n_cols >= ((int64_t)1 << 30)) return false;   // 32-bit byte offsets into x
    return m->opts.layout == SM_LAYOUT_SWEEP;
}

sm_status upload_sweep(sm_matrix *m, const int32_t *rp, const int32_t *col, const float *val) {
    std::vector<float> table;
    std::vector<uint8_t> ids;
    if (!codebook_ids(val, m->nnz, table, ids) || table.size() > 255) return SM_OK;   // not applicable
    SweepHost h;
    if (!sweep_build(rp, col, ids.data(), m->n_rows, h)) return SM_OK;
    std::vector<uint8_t>().swap(ids);
    SweepDev &d = m->plan.sw;
    SM_TRY_HIP(dev_alloc(&d.d_block_chunk, (int64_t)h.block_chunk.size(), m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_ent, std::max<int64_t>(1, h.n_chunks * 128), m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_table, 256, m->device_bytes));
    SM_TRY_HIP(hipMemset(d.d_table, 0, 256 * sizeof(float)));
    if (!table.empty())
        SM_TRY_HIP(hipMemcpy(d.d_table, table.data(), table.size() * 4, hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(d.d_block_chunk, h.block_chunk.data(), h.block_chunk.size() * 8, hipMemcpyHostToDevice));
    if (h.n_chunks)
        SM_TRY_HIP(hipMemcpy(d.d_ent, h.ent.data(), h.ent.size() * 4, hipMemcpyHostToDevice));
    d.table_size = (int32_t)table.size();
    d.n_chunks = h.n_chunks;
    d.n_blocks = h.n_blocks;
    return SM_OK;
}

bool want_ccsell(const sm_matrix *m) {
    if (m->opts.ccsell == 0 || m->opts.sell == 0) return false;
    if (m->nnz == 0 || m->n_rows == 0 || m->plan.xb.n_blocks > 0 || m->plan.n_relabel > 0 ||
        m->plan.sw.n_blocks > 0)
        return false;
    return m->opts.ccsell == 1 || m->n_cols >= ((int64_t)1 << 23);
}

sm_status upload_ccsell(sm_matrix *m, const int32_t *rp, const int32_t *col, const float *val) {
    const int32_t cl = m->opts.ccsell_chunk_log2 > 0 ? m->opts.ccsell_chunk_log2 : kCcDefaultChunkLog2;
    std::vector<float> table;
    std::vector<uint8_t> ids;
    const bool cb = m->opts.sell_codebook != 0 && cl <= 24 && codebook_ids(val, m->nnz, table, ids);
    if (!cb) std::vector<uint8_t>().swap(ids);
    CcsellHost h;
    // SM_CCSELL_ROWORDER (development A/B): units in row order instead of by length.
    const char *ro = dev_env("SM_CCSELL_ROWORDER");
    const bool by_length = !(ro && atoi(ro) == 1);
    if (!ccsell_build(rp, col, val, cb ? ids.data() : nullptr, m->n_rows, m->n_cols, cl, h, by_length))
        return SM_OK;   // not applicable: the sliced ELL serves the matrix
    std::vector<uint8_t>().swap(ids);
    if (h.n_slices == 0) return SM_OK;
    CcsellDev &d = m->plan.cc;
    SM_TRY_HIP(dev_alloc(&d.d_off, h.n_slices, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_len, h.n_slices, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_row, h.n_slices * kSellLanes, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_row_len, h.n_slices * kSellLanes, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_word, std::max<int64_t>(h.padded, 1), m->device_bytes));
    if (cb) {
        SM_TRY_HIP(dev_alloc(&d.d_table, 256, m->device_bytes));
        SM_TRY_HIP(hipMemset(d.d_table, 0, 256 * sizeof(float)));
        if (!table.empty())
            SM_TRY_HIP(hipMemcpy(d.d_table, table.data(), table.size() * 4, hipMemcpyHostToDevice));
        d.table_size = (int32_t)table.size();
    } else {
        SM_TRY_HIP(dev_alloc(&d.d_val, std::max<int64_t>(h.padded, 1), m->device_bytes));
        if (h.padded)
            SM_TRY_HIP(hipMemcpy(d.d_val, h.val.data(), (size_t)h.padded * 4, hipMemcpyHostToDevice));
    }
    SM_TRY_HIP(hipMemcpy(d.d_off, h.off.data(), h.off.size() * 8, hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(d.d_len, h.len.data(), h.len.size() * 4, hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(d.d_row, h.row.data(), h.row.size() * 4, hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(d.d_row_len, h.row_len.data(), h.row_len.size() * 2, hipMemcpyHostToDevice));
    if (h.padded)
        SM_TRY_HIP(hipMemcpy(d.d_word, h.word.data(), (size_t)h.padded * 4, hipMemcpyHostToDevice));
    d.n_chunks = h.n_chunks;
    d.chunk_log2 = h.chunk_log2;
    d.chunk_slice = std::move(h.chunk_slice);
    d.n_slices = h.n_slices;
    return SM_OK;
}

// The reference's stream on the device (native.hip, SM_ALGO_NATIVE): each panel's run
// padded to start at a multiple of 16 bytes with (delta 0, id T) fillers, which the
// decode skips like the reference's own fillers -- so every 16-entry load is aligned.
sm_status upload_native(sm_matrix *m) {
    if (!m->has_ref || m->panel_col_off.empty() || m->table_size <= 0) return SM_OK;
    if (m->s_rows >= ((int64_t)1 << 23)) return SM_OK;   // in-panel offsets in int32
    const size_t P = m->panel_col_off.size();
    const size_t P_all = (size_t)((m->s_cols + 255) / 256);
    std::vector<uint8_t> pos, val;
    // Panels with entries first, then every 256-column block without one (an empty run):
    // a beta != 1 launch covers them all, since the kernel applies beta to the columns
    // it owns and the reference scales all of C (sparse-matrix.cc:149-151).
    std::vector<int64_t> beg(P, 0), end(P, 0);
    std::vector<int32_t> cols(m->panel_col_off.begin(), m->panel_col_off.end());
    {
        std::vector<char> has(P_all, 0);
        for (size_t p = 0; p < P; p++) has[(size_t)m->panel_col_off[p] / 256] = 1;
        for (size_t q = 0; q < P_all; q++)
            if (!has[q]) cols.push_back((int32_t)(q * 256));
        beg.resize(cols.size(), 0);
        end.resize(cols.size(), 0);
    }
    pos.reserve(m->pos.size() + 16 * P);
    val.reserve(m->pos.size() + 16 * P);
    for (size_t p = 0; p < P; p++) {
        while (pos.size() % 16) { pos.push_back(0); val.push_back((uint8_t)m->table_size); }
        beg[p] = (int64_t)pos.size();
        pos.insert(pos.end(), m->pos.begin() + m->panel_begin[p], m->pos.begin() + m->panel_end[p]);
        val.insert(val.end(), m->val.begin() + m->panel_begin[p], m->val.begin() + m->panel_end[p]);
        end[p] = (int64_t)pos.size();
    }
    NativeDev &d = m->plan.nat;
    SM_TRY_HIP(dev_alloc(&d.d_pos, (int64_t)pos.size() + 16, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_val, (int64_t)val.size() + 16, m->device_bytes));
    const size_t Pc = cols.size();
    SM_TRY_HIP(dev_alloc(&d.d_beg, (int64_t)Pc, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_end, (int64_t)Pc, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_col, (int64_t)Pc, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&d.d_table, 256, m->device_bytes));
    SM_TRY_HIP(hipMemset(d.d_table, 0, 256 * sizeof(float)));
    SM_TRY_HIP(hipMemcpy(d.d_pos, pos.data(), pos.size(), hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(d.d_val, val.data(), val.size(), hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(d.d_beg, beg.data(), Pc * 8, hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(d.d_end, end.data(), Pc * 8, hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(d.d_col, cols.data(), Pc * 4, hipMemcpyHostToDevice));
    SM_TRY_HIP(hipMemcpy(d.d_table, m->table.data(), (size_t)m->table_size * 4, hipMemcpyHostToDevice));
    d.table_size = m->table_size;
    d.s_rows = m->s_rows;
    d.s_cols = m->s_cols;
    d.n_panels = (int32_t)P;
    d.n_all = (int32_t)Pc;
    // Batch metadata of the two-kernel form: the carry before each batch and the live
    // entries of each (batch, group) -- derived from the stream once, as the panel bounds are.
    std::vector<int32_t> pbatch(Pc + 1, 0), boff;
    std::vector<NatBatch> bmeta;
    int64_t live_total = 0;
    for (size_t p = 0; p < Pc; p++) {
        pbatch[p] = (int32_t)bmeta.size();
        int32_t carry = 0;
        for (int64_t e0 = beg[p]; e0 < end[p]; e0 += kNatBatchEntries) {
            const int64_t e1 = std::min<int64_t>(end[p], e0 + kNatBatchEntries);
            bmeta.push_back(NatBatch{e0, (int32_t)(e1 - e0), carry});
            int64_t live[4] = {0, 0, 0, 0};
            for (int64_t e = e0; e < e1; e++) {
                carry += pos[(size_t)e];
                if (val[(size_t)e] < m->table_size) live[(carry & 255) >> 6]++;
            }
            for (int g = 0; g < 4; g++) {
                boff.push_back((int32_t)live_total);
                live_total += live[g];
            }
        }
        d.max_panel_batches = std::max<int32_t>(d.max_panel_batches, (int32_t)bmeta.size() - pbatch[p]);
    }
    pbatch[Pc] = (int32_t)bmeta.size();
    d.n_batches = (int32_t)bmeta.size();
    if (live_total >= ((int64_t)1 << 31)) return SM_OK;   // fused kernel only
    if (d.n_batches > 0 && d.max_panel_batches > kNatFusedBatches) {
        SM_TRY_HIP(dev_alloc(&d.d_pbatch, (int64_t)Pc + 1, m->device_bytes));
        SM_TRY_HIP(dev_alloc(&d.d_bmeta, (int64_t)d.n_batches, m->device_bytes));
        SM_TRY_HIP(dev_alloc(&d.d_boff, (int64_t)d.n_batches * 4, m->device_bytes));
        SM_TRY_HIP(dev_alloc(&d.d_lists, std::max<int64_t>(live_total, 1), m->device_bytes));
        SM_TRY_HIP(dev_alloc(&d.d_hdr, (int64_t)d.n_batches * 256, m->device_bytes));
        SM_TRY_HIP(hipMemcpy(d.d_pbatch, pbatch.data(), (Pc + 1) * 4, hipMemcpyHostToDevice));
        SM_TRY_HIP(hipMemcpy(d.d_bmeta, bmeta.data(), bmeta.size() * sizeof(NatBatch), hipMemcpyHostToDevice));
        SM_TRY_HIP(hipMemcpy(d.d_boff, boff.data(), boff.size() * 4, hipMemcpyHostToDevice));
    }
    return SM_OK;
}

// Skewed graphs (column relabeling built, e.g. R-MAT): the hottest
// relabeled columns [0, H) hold a large share of the terms in few columns, so they go
// through the codebook band kernel with their x staged in LDS (kernels_band2.hip) --
// no gathers -- and the sliced ELL gathers only the rest.  A row then adds its hot
// terms (in relabeled column order) before its cold ones (stored order): within the
// Sum|terms| bound, deterministic.  Opt-in only (hot_cols > 0 sets H; 0 and -1 never):
// measured on R-MAT scale 24 the split loses -- 2.71 ms at H = 32768, 2.16 ms at 8192,
// 4.55 ms at 131072 against 1.66 ms for the codebook sliced ELL alone (the band pass
// over 2^24 rows costs ~1.4 ms by itself; profiles/r03_rmat24_layout_ab.txt).
sm_status upload_sell_layouts(sm_matrix *m, const int32_t *rp, const int32_t *col, const float *val) {
    Plan &p = m->plan;
    const int64_t H0 = m->opts.hot_cols > 0 ? m->opts.hot_cols : 0;
    const bool try_hot = p.n_relabel > 0 && H0 > 0 && H0 < m->n_cols;
    if (!try_hot) return upload_sell(m, rp, col, val);
    const int64_t nnz = m->nnz, nr = m->n_rows;
    std::vector<int32_t> rcol((size_t)nnz);
    SM_TRY_HIP(hipMemcpy(rcol.data(), p.d_rcol, (size_t)nnz * 4, hipMemcpyDeviceToHost));
    int64_t hot = 0;
    for (int64_t e = 0; e < nnz; e++) hot += rcol[(size_t)e] < H0;
    // Split every row into its hot part (sorted by relabeled column: the bands need
    // ascending columns) and its cold part (stored order).
    std::vector<int32_t> rph((size_t)nr + 1, 0), rpc((size_t)nr + 1, 0);
    std::vector<int32_t> ch((size_t)hot), cc((size_t)(nnz - hot));
    std::vector<float> vh((size_t)hot), vc((size_t)(nnz - hot));
    std::vector<std::pair<int32_t, float>> tmp;
    int64_t oh = 0, oc = 0;
    for (int64_t r = 0; r < nr; r++) {
        tmp.clear();
        for (int32_t e = rp[r]; e < rp[r + 1]; e++) {
            if (rcol[(size_t)e] < H0) {
                tmp.push_back({rcol[(size_t)e], val[e]});
            } else {
                cc[(size_t)oc] = rcol[(size_t)e];
                vc[(size_t)oc++] = val[e];
            }
        }
        std::sort(tmp.begin(), tmp.end(),
                  [](const std::pair<int32_t, float> &a, const std::pair<int32_t, float> &b) { return a.first < b.first; });
        for (const auto &t : tmp) {
            ch[(size_t)oh] = t.first;
            vh[(size_t)oh++] = t.second;
        }
        rph[(size_t)r + 1] = (int32_t)oh;
        rpc[(size_t)r + 1] = (int32_t)oc;
    }
    std::vector<int32_t>().swap(rcol);
    sm_status st = build_band2(m, p.hot, nr, H0, hot, rph.data(), ch.data(), vh.data(), kXbCband,
                               0, 0, true);
    if (st != SM_OK) return st;
    if (p.hot.n_blocks == 0 || p.hot.kind != kXbCband) {   // not applicable: sell serves all terms
        free_xband_dev(p.hot);
        return upload_sell(m, rp, col, val);
    }
    p.hot_cols = (int32_t)H0;
    std::vector<int32_t>().swap(ch);
    std::vector<float>().swap(vh);
    return upload_sell(m, rpc.data(), cc.data(), vc.data(), nnz - hot, true);
}

sm_status upload_plan(sm_matrix *m, const int32_t *rp_host) {
    PlanHost ph;
    int32_t tile = tile_nnz_setting(m);
    // Power-law rows (longest row > 64x the mean, e.g. R-MAT): 2048-term tiles
    // balance the workgroups better -- R-MAT scale 24: 2.34 ms vs 2.43 ms at 4096
    // (profiles/r01_rmat24_sweep.txt).  tile_nnz overrides.
    if (m->opts.tile_nnz == 0 && m->n_rows > 0) {
        int64_t longest = 0;
        for (int64_t r = 0; r < m->n_rows; r++)
            longest = std::max<int64_t>(longest, (int64_t)rp_host[r + 1] - rp_host[r]);
        if ((double)longest > 64.0 * (double)m->nnz / (double)m->n_rows) tile = 2048;
    }
    plan_rows(rp_host, m->n_rows, tile, kTileRows, kLongChunk, kSerialRowMax, ph);
    std::vector<Tile> tiles(ph.tiles.size());
    for (size_t i = 0; i < tiles.size(); i++)
        tiles[i] = Tile{ph.tiles[i].r0, ph.tiles[i].r1, ph.tiles[i].flags, 0};
    std::vector<Chunk> chunks(ph.chunks.size());
    for (size_t i = 0; i < chunks.size(); i++)
        chunks[i] = Chunk{ph.chunks[i].lr, ph.chunks[i].begin, ph.chunks[i].end, 0};
    Plan &p = m->plan;
    p.tile_nnz = tile;
    p.n_tiles = (int32_t)tiles.size();
    p.n_long = (int32_t)ph.long_rows.size();
    p.n_chunks = (int32_t)chunks.size();
    p.max_row_nnz = ph.max_row_nnz;
    p.avg_row_nnz = ph.avg_row_nnz;
    SM_TRY_HIP(dev_alloc(&p.d_tiles, p.n_tiles, m->device_bytes));
    if (m->n_rows > 0 && m->nnz > 0) {   // merge path (SM_ALGO_MERGE): slice corners, 32 B records
        const int64_t nb = merge_blocks(m->n_rows, m->nnz);
        std::vector<int32_t> corners;
        merge_corners(rp_host, m->n_rows, m->nnz, corners);
        SM_TRY_HIP(dev_alloc(&p.d_merge, nb, m->device_bytes));
        SM_TRY_HIP(dev_alloc(&p.d_merge_corner, nb + 1, m->device_bytes));
        SM_TRY_HIP(hipMemcpy(p.d_merge_corner, corners.data(), corners.size() * 4, hipMemcpyHostToDevice));
    }
    SM_TRY_HIP(dev_alloc(&p.d_chunks, p.n_chunks, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&p.d_partials, p.n_chunks, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&p.d_long_rows, p.n_long, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&p.d_long_ptr, p.n_long + 1, m->device_bytes));
    if (p.n_tiles)
        SM_TRY_HIP(hipMemcpy(p.d_tiles, tiles.data(), tiles.size() * sizeof(Tile), hipMemcpyHostToDevice));
    if (p.n_chunks)
        SM_TRY_HIP(hipMemcpy(p.d_chunks, chunks.data(), chunks.size() * sizeof(Chunk), hipMemcpyHostToDevice));
    if (p.n_long) {
        SM_TRY_HIP(hipMemcpy(p.d_long_rows, ph.long_rows.data(), ph.long_rows.size() * 4, hipMemcpyHostToDevice));
        SM_TRY_HIP(hipMemcpy(p.d_long_ptr, ph.long_ptr.data(), ph.long_ptr.size() * 4, hipMemcpyHostToDevice));
    }
    return SM_OK;
}

// Allocate the CSR arrays (col/val carry a zeroed tail of kPadElems for the
// aligned 16-byte loads of the stream kernel).
sm_status alloc_csr(sm_matrix *m) {
    SM_TRY_HIP(dev_alloc(&m->d_row_ptr, m->n_rows + 1, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&m->d_col, m->nnz + kPadElems, m->device_bytes));
    SM_TRY_HIP(dev_alloc(&m->d_val, m->nnz + kPadElems, m->device_bytes));
    SM_TRY_HIP(hipMemset(m->d_col + m->nnz, 0, kPadElems * sizeof(int32_t)));
    SM_TRY_HIP(hipMemset(m->d_val + m->nnz, 0, kPadElems * sizeof(float)));
    return SM_OK;
}

sm_status check_sizes(int64_t n_rows, int64_t n_cols, int64_t nnz) {
    if (n_rows < 0 || n_cols < 0 || nnz < 0) return fail(SM_ERR_INVALID_ARG, "negative size");
    if (n_rows >= kI32Max || n_cols >= kI32Max || nnz >= kI32Max - kPadElems)
        return fail(SM_ERR_TOO_LARGE, "rows/cols/nnz must be < 2^31 (int32 indexing)");
    return SM_OK;
}

sm_status check_device(int32_t device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return fail(SM_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= n) return fail(SM_ERR_INVALID_ARG, "device %d out of range", device);
    return SM_OK;
}

// Common tail of the host-CSR constructors.
sm_status finish_from_host_csr(sm_matrix *m, const int32_t *rp, const int32_t *col,
                               const float *val) {
    sm_status st = alloc_csr(m);
    if (st != SM_OK) return st;
    SM_TRY_HIP(hipMemcpy(m->d_row_ptr, rp, (size_t)(m->n_rows + 1) * 4, hipMemcpyHostToDevice));
    if (m->nnz) {
        SM_TRY_HIP(hipMemcpy(m->d_col, col, (size_t)m->nnz * 4, hipMemcpyHostToDevice));
        SM_TRY_HIP(hipMemcpy(m->d_val, val, (size_t)m->nnz * 4, hipMemcpyHostToDevice));
    }
    sm_status st2 = upload_plan(m, rp);
    if (st2 == SM_OK && want_xband(m)) st2 = upload_xband(m, rp, col, val, xband_kind_setting(m));
    if (st2 == SM_OK && want_sweep(m)) st2 = upload_sweep(m, rp, col, val);
    if (st2 == SM_OK && want_relabel_size(m)) st2 = upload_relabel(m, col);
    if (st2 == SM_OK && want_ccsell(m)) st2 = upload_ccsell(m, rp, col, val);
    if (st2 == SM_OK && want_sell(m)) st2 = upload_sell_layouts(m, rp, col, val);
    if (st2 == SM_OK && want_merge_stage(m)) st2 = upload_merge_stage(m, rp, col, val);
    if (st2 == SM_OK && want_exact_sell(m)) st2 = upload_exact_sell(m, rp, col, val);
    return st2;
}

std::unique_ptr<sm_matrix> new_matrix(int32_t device, const sm_build_opts *opts = nullptr) {
    std::unique_ptr<sm_matrix> m(new sm_matrix());
    m->device = device;
    m->opts = resolve_opts(opts);
    return m;
}

}  // namespace

namespace {
// Launches that use the matrix's scratch (sm_internal.h: scratch_ready) run one after
// the other on the device: the stream waits for the previous such launch's event, and
// records it after its own (not while the stream is being captured into a graph).
template <class F>
hipError_t with_scratch(const sm_matrix *m, hipStream_t s, bool needed, F &&launch) {
    if (!needed) return launch();
    std::lock_guard<std::mutex> lk(m->scratch_mu);
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess) cs = hipStreamCaptureStatusNone;
    const bool ordered = cs == hipStreamCaptureStatusNone;
    hipError_t e = hipSuccess;
    if (ordered && !m->scratch_ready) e = hipEventCreateWithFlags(&m->scratch_ready, hipEventDisableTiming);
    if (ordered && e == hipSuccess && m->scratch_recorded) e = hipStreamWaitEvent(s, m->scratch_ready, 0);
    if (e != hipSuccess) return e;
    e = launch();
    if (ordered) {   // whatever was queued (also on a failed launch) uses the scratch
        const hipError_t er = hipEventRecord(m->scratch_ready, s);
        if (er == hipSuccess) m->scratch_recorded = true;
        if (e == hipSuccess) e = er;
    }
    return e;
}

bool native_scratch(const NativeDev &nd) { return nd.d_lists && nd.max_panel_batches > kNatFusedBatches; }
}  // namespace

namespace {
// FNV-1a over device arrays (sm_layout_digest).
struct Fnv {
    uint64_t h = 1469598103934665603ull;
    void add(const void *p, size_t n) {
        const uint8_t *b = static_cast<const uint8_t *>(p);
        for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
    }
};
template <class T>
sm_status fnv_dev(Fnv &f, const T *d, int64_t n) {
    if (!d || n <= 0) return SM_OK;
    std::vector<T> h((size_t)n);
    const hipError_t e = hipMemcpy(h.data(), d, (size_t)n * sizeof(T), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_fail(e, "sm_layout_digest");
    f.add(h.data(), h.size() * sizeof(T));
    return SM_OK;
}
}  // namespace

extern "C" {

const char *sm_version(void) { return "sparsematrix_amd 0.2 (gfx950)"; }

const char *sm_status_string(sm_status s) {
    switch (s) {
    case SM_OK: return "ok";
    case SM_ERR_INVALID_ARG: return "invalid argument";
    case SM_ERR_OUT_OF_MEMORY: return "out of memory";
    case SM_ERR_HIP: return "HIP runtime error";
    case SM_ERR_NOT_SUPPORTED: return "not supported";
    case SM_ERR_TOO_LARGE: return "too large for int32 indexing";
    case SM_ERR_INVALID_MATRIX: return "invalid matrix";
    case SM_ERR_NO_DEVICE: return "no HIP device";
    }
    return "unknown status";
}

const char *sm_last_error(void) { return g_err.c_str(); }

sm_status sm_device_count(int32_t *count) {
    if (!count) return fail(SM_ERR_INVALID_ARG, "count is null");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return n ? SM_OK : fail(SM_ERR_NO_DEVICE, "no HIP device visible");
}

void sm_destroy(sm_matrix *m) {
    if (!m) return;
    free_device(m);
    delete m;
}

sm_status sm_create_from_dense_index(const uint8_t *index, int32_t rows, int32_t cols,
                                     int32_t stride, const float *table, int32_t table_size,
                                     sm_trans trans, int32_t device, sm_matrix **out) {
    if (!out) return fail(SM_ERR_INVALID_ARG, "out is null");
    *out = nullptr;
    if (table_size < 0 || table_size > 255)
        return fail(SM_ERR_INVALID_ARG, "table_size %d not in [0, 255]", table_size);
    if (rows < 0 || cols < 0 || stride < cols)
        return fail(SM_ERR_INVALID_ARG, "bad shape rows=%d cols=%d stride=%d", rows, cols, stride);
    if (trans != SM_NO_TRANS && trans != SM_TRANS) return fail(SM_ERR_INVALID_ARG, "bad trans");
    if (table_size > 0 && rows > 0 && cols > 0 && (!index || !table))
        return fail(SM_ERR_INVALID_ARG, "null index/table");
    sm_status st = check_device(device);
    if (st != SM_OK) return st;
    DeviceGuard g(device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");

    EncodeResult er;
    if (table_size > 0 && rows > 0 && cols > 0) {
        if (encode_dense_index(index, rows, cols, stride, table, table_size, trans == SM_TRANS, er))
            return fail(SM_ERR_INVALID_ARG, "encode failed");
    } else if (table_size > 0) {
        // degenerate shape: the reference still records rows_/cols_ (:63-64, :96-97)
        er.s_rows = trans == SM_TRANS ? cols : rows;
        er.s_cols = trans == SM_TRANS ? rows : cols;
        er.table.assign(table, table + table_size);
        er.table.push_back(0.0f);
        er.table_size = table_size;
        er.row_ptr.assign((size_t)er.s_cols + 1, 0);
    } else {
        er.row_ptr.assign(1, 0);   // val_table_size == 0: empty 0 x 0 (:26)
    }
    const int64_t nnz = er.row_ptr.back();
    st = check_sizes(er.s_cols, er.s_rows, nnz);
    if (st != SM_OK) return st;

    auto m = new_matrix(device);
    m->n_rows = er.s_cols;
    m->n_cols = er.s_rows;
    m->nnz = nnz;
    m->s_rows = er.s_rows;
    m->s_cols = er.s_cols;
    m->has_ref = true;   // the reference encoding exists (possibly empty)
    m->from_index = true;
    m->table_size = er.table_size;
    m->table = std::move(er.table);
    m->pos = std::move(er.pos);
    m->val = std::move(er.val_id);
    m->panel_row_off = std::move(er.panel_row_off);
    m->panel_col_off = std::move(er.panel_col_off);
    m->panel_begin = std::move(er.panel_begin);
    m->panel_end = std::move(er.panel_end);
    std::vector<int32_t> rp32(er.row_ptr.size());
    for (size_t i = 0; i < rp32.size(); i++) rp32[i] = (int32_t)er.row_ptr[i];
    st = finish_from_host_csr(m.get(), rp32.data(), er.col.data(), er.val.data());
    if (st == SM_OK) st = upload_native(m.get());
    if (st != SM_OK) {
        free_device(m.get());
        return st;
    }
    *out = m.release();
    return SM_OK;
}

// CopyForm's scan on the device (encode_dev.hip): count, host prefix sum, fill, then the
// device-CSR constructor (validation, plans, band layout).  Same CSR as the host
// encoder, bit for bit, and the same reference stream (refenc_dev.hip, from the ids).
sm_status sm_create_from_dense_index_device(const uint8_t *d_index, int32_t rows, int32_t cols,
                                            int32_t stride, const float *table,
                                            int32_t table_size, sm_trans trans, int32_t device,
                                            sm_stream stream, sm_matrix **out) {
    if (!out) return fail(SM_ERR_INVALID_ARG, "out is null");
    *out = nullptr;
    if (table_size < 0 || table_size > 255)
        return fail(SM_ERR_INVALID_ARG, "table_size %d not in [0, 255]", table_size);
    if (rows < 0 || cols < 0 || stride < cols)
        return fail(SM_ERR_INVALID_ARG, "bad shape rows=%d cols=%d stride=%d", rows, cols, stride);
    if (trans != SM_NO_TRANS && trans != SM_TRANS) return fail(SM_ERR_INVALID_ARG, "bad trans");
    if (table_size == 0 || rows == 0 || cols == 0)   // nothing to scan: the host rules apply
        return sm_create_from_dense_index(nullptr, rows, cols, stride, table, table_size, trans,
                                          device, out);
    if (!d_index || !table) return fail(SM_ERR_INVALID_ARG, "null index/table");
    sm_status st = check_device(device);
    if (st != SM_OK) return st;
    DeviceGuard g(device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    hipStream_t s = (hipStream_t)stream;
    const bool tr = trans == SM_TRANS;
    const uint8_t T = (uint8_t)table_size;
    const int64_t nb = tr ? rows : cols;    // rows of B = columns of S
    const int64_t kb = tr ? cols : rows;    // columns of B = rows of S
    // NoTrans: index rows split in chunks so the count/fill grids fill the chip.
    const int32_t chunk_rows = tr ? rows : std::max<int32_t>(256, (rows + 63) / 64);
    const int32_t n_chunks = tr ? 1 : (rows + chunk_rows - 1) / chunk_rows;
    const int64_t n_cnt = tr ? nb : (int64_t)n_chunks * nb;
    std::vector<int32_t> cnt((size_t)n_cnt);
    int32_t *d_cnt = nullptr, *d_offs = nullptr, *d_rp = nullptr, *d_col = nullptr;
    float *d_table = nullptr, *d_val = nullptr;
    uint8_t *d_ids = nullptr;
    int64_t scratch = 0;
    auto cleanup = [&]() {
        (void)hipFree(d_cnt); (void)hipFree(d_offs); (void)hipFree(d_rp);
        (void)hipFree(d_col); (void)hipFree(d_val); (void)hipFree(d_table); (void)hipFree(d_ids);
    };
    hipError_t e = dev_alloc(&d_cnt, n_cnt, scratch);
    if (e == hipSuccess)
        e = launch_encode_count(d_index, rows, cols, stride, tr, chunk_rows, n_chunks, T, d_cnt, s);
    if (e == hipSuccess)
        e = hipMemcpyAsync(cnt.data(), d_cnt, (size_t)n_cnt * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) { cleanup(); return hip_fail(e, "dense index count"); }
    // Prefix sums: row_ptr over B rows; per (chunk, row) start offsets.
    std::vector<int64_t> rp64((size_t)nb + 1, 0);
    std::vector<int32_t> offs((size_t)n_cnt);
    for (int64_t j = 0; j < nb; j++) {
        int64_t t = 0;
        for (int32_t ch = 0; ch < n_chunks; ch++) t += cnt[(size_t)(ch * nb + j)];
        rp64[(size_t)j + 1] = rp64[(size_t)j] + t;
    }
    const int64_t nnz = rp64[(size_t)nb];
    st = check_sizes(nb, kb, nnz);
    if (st != SM_OK) { cleanup(); return st; }
    for (int64_t j = 0; j < nb; j++) {
        int64_t o = rp64[(size_t)j];
        for (int32_t ch = 0; ch < n_chunks; ch++) {
            offs[(size_t)(ch * nb + j)] = (int32_t)o;
            o += cnt[(size_t)(ch * nb + j)];
        }
    }
    std::vector<int32_t> rp32(rp64.begin(), rp64.end());
    std::vector<float> tb(table, table + table_size);
    tb.push_back(0.0f);
    e = dev_alloc(&d_offs, n_cnt, scratch);
    if (e == hipSuccess) e = dev_alloc(&d_rp, nb + 1, scratch);
    if (e == hipSuccess) e = dev_alloc(&d_table, (int64_t)tb.size(), scratch);
    if (e == hipSuccess) e = dev_alloc(&d_col, std::max<int64_t>(nnz, 1), scratch);
    if (e == hipSuccess) e = dev_alloc(&d_val, std::max<int64_t>(nnz, 1), scratch);
    if (e == hipSuccess) e = dev_alloc(&d_ids, std::max<int64_t>(nnz, 1), scratch);
    if (e == hipSuccess)
        e = hipMemcpyAsync(d_offs, offs.data(), (size_t)n_cnt * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
        e = hipMemcpyAsync(d_rp, rp32.data(), rp32.size() * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
        e = hipMemcpyAsync(d_table, tb.data(), tb.size() * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
        e = launch_encode_fill(d_index, rows, cols, stride, tr, chunk_rows, n_chunks, T,
                               tr ? d_rp : d_offs, d_table, d_col, d_val, d_ids, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);   // host vectors above go out of scope
    if (e != hipSuccess) { cleanup(); return hip_fail(e, "dense index fill"); }
    sm_build_opts o;   // the CopyForm path: SM_ALGO_EXACT keeps a reference-order kernel
    sm_build_opts_init(&o);
    o.exact_sell = 1;
    st = sm_create_from_csr_device_ex(nb, kb, nnz, d_rp, d_col, d_val, device, stream, &o, out);
    if (st == SM_OK) {
        sm_matrix *m = *out;
        m->from_index = true;
        m->table_size = table_size;
        m->table = std::move(tb);
        // The reference stream from the index's own ids (refenc_dev.hip), as the host
        // constructor keeps it; S rows >= 2^23 (the reference's int32 offsets) keep none.
        EncodeResult er;
        hipError_t he = hipSuccess;
        const int rc = encode_csr_ref_device(d_rp, d_col, d_val, d_ids, nb, kb, nnz, table, table_size, er, s, he);
        if (rc == 0) {
            m->has_ref = true;
            m->pos = std::move(er.pos);
            m->val = std::move(er.val_id);
            m->panel_row_off = std::move(er.panel_row_off);
            m->panel_col_off = std::move(er.panel_col_off);
            m->panel_begin = std::move(er.panel_begin);
            m->panel_end = std::move(er.panel_end);
            st = upload_native(m);
        } else if (rc != -4) {
            st = rc == -5 ? hip_fail(he, "dense index reference stream")
                          : fail(SM_ERR_INVALID_ARG, "dense index reference stream (%d)", rc);
        }
        if (st != SM_OK) {
            sm_destroy(m);
            *out = nullptr;
        }
    }
    cleanup();
    return st;
}

void sm_build_opts_init(sm_build_opts *o) {
    if (!o) return;
    memset(o, 0, sizeof(*o));
    o->struct_size = (int32_t)sizeof(*o);
    o->layout = SM_LAYOUT_AUTO;
    o->sell = -1;
    o->sell_codebook = -1;
    o->relabel = -1;
    o->ccsell = -1;
}

sm_status sm_create_from_csr(int64_t n_rows, int64_t n_cols, int64_t nnz, const int32_t *row_ptr,
                             const int32_t *col_idx, const float *val, int32_t device,
                             sm_matrix **out) {
    return sm_create_from_csr_ex(n_rows, n_cols, nnz, row_ptr, col_idx, val, device, nullptr, out);
}

sm_status sm_create_from_csr_ex(int64_t n_rows, int64_t n_cols, int64_t nnz,
                                const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                                int32_t device, const sm_build_opts *opts, sm_matrix **out) {
    if (!out) return fail(SM_ERR_INVALID_ARG, "out is null");
    *out = nullptr;
    sm_status st = check_opts(opts);
    if (st != SM_OK) return st;
    st = check_sizes(n_rows, n_cols, nnz);
    if (st != SM_OK) return st;
    if (!row_ptr || (nnz > 0 && (!col_idx || !val)))
        return fail(SM_ERR_INVALID_ARG, "null CSR array");
    // host validation: monotone row_ptr, columns in range
    if (row_ptr[0] != 0 || row_ptr[n_rows] != nnz)
        return fail(SM_ERR_INVALID_MATRIX, "row_ptr[0] must be 0 and row_ptr[n] == nnz");
    for (int64_t r = 0; r < n_rows; r++)
        if (row_ptr[r + 1] < row_ptr[r])
            return fail(SM_ERR_INVALID_MATRIX, "row_ptr decreases at row %lld", (long long)r);
    for (int64_t e = 0; e < nnz; e++)
        if (col_idx[e] < 0 || col_idx[e] >= n_cols)
            return fail(SM_ERR_INVALID_MATRIX, "col_idx[%lld] = %d out of range", (long long)e,
                        col_idx[e]);
    st = check_device(device);
    if (st != SM_OK) return st;
    DeviceGuard g(device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    auto m = new_matrix(device, opts);
    m->n_rows = n_rows;
    m->n_cols = n_cols;
    m->nnz = nnz;
    m->s_rows = n_cols;
    m->s_cols = n_rows;
    st = finish_from_host_csr(m.get(), row_ptr, col_idx, val);
    if (st != SM_OK) {
        free_device(m.get());
        return st;
    }
    *out = m.release();
    return SM_OK;
}

sm_status sm_create_from_csr_device(int64_t n_rows, int64_t n_cols, int64_t nnz,
                                    const int32_t *d_row_ptr, const int32_t *d_col_idx,
                                    const float *d_val, int32_t device, sm_stream stream,
                                    sm_matrix **out) {
    return sm_create_from_csr_device_ex(n_rows, n_cols, nnz, d_row_ptr, d_col_idx, d_val, device,
                                        stream, nullptr, out);
}

sm_status sm_create_from_csr_device_ex(int64_t n_rows, int64_t n_cols, int64_t nnz,
                                       const int32_t *d_row_ptr, const int32_t *d_col_idx,
                                       const float *d_val, int32_t device, sm_stream stream,
                                       const sm_build_opts *opts, sm_matrix **out) {
    if (!out) return fail(SM_ERR_INVALID_ARG, "out is null");
    *out = nullptr;
    sm_status st = check_opts(opts);
    if (st != SM_OK) return st;
    st = check_sizes(n_rows, n_cols, nnz);
    if (st != SM_OK) return st;
    if (!d_row_ptr || (nnz > 0 && (!d_col_idx || !d_val)))
        return fail(SM_ERR_INVALID_ARG, "null CSR array");
    st = check_device(device);
    if (st != SM_OK) return st;
    DeviceGuard g(device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    hipStream_t s = (hipStream_t)stream;
    auto m = new_matrix(device, opts);
    m->n_rows = n_rows;
    m->n_cols = n_cols;
    m->nnz = nnz;
    m->s_rows = n_cols;
    m->s_cols = n_rows;
    st = alloc_csr(m.get());
    if (st != SM_OK) { free_device(m.get()); return st; }
    hipError_t e = hipMemcpyAsync(m->d_row_ptr, d_row_ptr, (size_t)(n_rows + 1) * 4,
                                  hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess && nnz) {
        e = hipMemcpyAsync(m->d_col, d_col_idx, (size_t)nnz * 4, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess)
            e = hipMemcpyAsync(m->d_val, d_val, (size_t)nnz * 4, hipMemcpyDeviceToDevice, s);
    }
    int32_t *d_flag = nullptr;
    if (e == hipSuccess) e = hipMalloc((void **)&d_flag, sizeof(int32_t));
    if (e == hipSuccess) e = hipMemsetAsync(d_flag, 0, sizeof(int32_t), s);
    if (e == hipSuccess)
        e = launch_validate((int32_t)n_rows, (int32_t)n_cols, (int32_t)nnz, m->d_row_ptr,
                            m->d_col, d_flag, s);
    int32_t flag = 0;
    std::vector<int32_t> rp((size_t)n_rows + 1);
    if (e == hipSuccess) e = hipMemcpyAsync(&flag, d_flag, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess)
        e = hipMemcpyAsync(rp.data(), m->d_row_ptr, rp.size() * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(d_flag);
    if (e != hipSuccess) {
        free_device(m.get());
        return hip_fail(e, "sm_create_from_csr_device");
    }
    if (flag) {
        free_device(m.get());
        return fail(SM_ERR_INVALID_MATRIX, "device CSR failed validation (flags 0x%x)", flag);
    }
    st = upload_plan(m.get(), rp.data());
    const bool xband = want_xband(m.get());
    // The column relabeling and the sorted sliced ELL on the device (builddev.hip) where they
    // are all this matrix wants: no band layout, sweep, hot split, windowed sort or exact sliced
    // ELL, and no column-chunked ELL once the relabeling is decided (its builder runs on the
    // host).  R-MAT 24: the host path took 5.4 s.
    bool dev_done = false;
    const bool dev_ok = st == SM_OK && m->opts.host_build == 0 && !want_sweep(m.get()) && m->opts.hot_cols <= 0 &&
                        m->opts.sell_sigma == 0 && m->opts.sell_streams <= 1 && m->opts.exact_sell != 1;
    // The gathered chunk bands on the device (builddev_gcb.hip; config 5: 15 s on the host path).
    // Declined (a row's columns not ascending, size limits): the host path below decides.
    if (dev_ok && xband && xband_kind_setting(m.get()) == kXbGcb) {
        hipError_t eb = hipSuccess;
        int rows_log2 = 0;
        int32_t slabs = 1;
        gcb_geometry(m.get(), rows_log2, slabs);
        GcbHost meta;
        const int rc = devbuild_gcb(m.get(), rows_log2, slabs, kGcbMaxWindow, meta, s, eb);
        if (rc < 0) st = hip_fail(eb, "device gcb builder");
        else if (rc == 0) {
            st = gcb_finish(m.get(), meta);
            dev_done = st == SM_OK;
        }
    }
    if (dev_ok && !xband) {
        hipError_t eb = hipSuccess;
        int rc = 0;
        if (want_relabel_size(m.get())) rc = devbuild_relabel(m.get(), m->opts.relabel != 1, s, eb);
        if (rc == 0 && !want_ccsell(m.get())) {
            if (want_sell(m.get())) {
                const int32_t max_len = m->opts.sell_max_len > 0 ? m->opts.sell_max_len : kSellMaxLen;
                rc = devbuild_sell(m.get(), max_len, m->opts.sell_codebook != 0, s, eb);
            }
            dev_done = rc == 0;
        }
        if (rc != 0) st = hip_fail(eb, "device layout builder");
    }
    // The merge path's staging copy (sm_build_opts.merge_stage) after a device build too
    // (R-MAT 24: 7.7 s on the host path).
    if (st == SM_OK && dev_done && want_merge_stage(m.get())) {
        hipError_t eb = hipSuccess;
        if (devbuild_merge_stage(m.get(), s, eb) < 0) st = hip_fail(eb, "device merge staging builder");
    }
    const bool maybe_sell = m->opts.sell != 0 && nnz > 0;
    // The band / sell builders run on the host (band2.cpp, xband.cpp, sell.cpp): the
    // columns come down for any of them, the values only for the layout that stores
    // them (4 + 4 bytes per term over PCIe once, at creation).
    if (st == SM_OK && !dev_done &&
        (xband || want_relabel_size(m.get()) || maybe_sell || want_sweep(m.get()) || want_merge_stage(m.get()))) {
        std::vector<int32_t> ch((size_t)nnz);
        std::vector<float> vh;
        auto values = [&]() -> sm_status {
            if (vh.size() == (size_t)nnz) return SM_OK;
            vh.resize((size_t)nnz);
            const hipError_t ev = hipMemcpy(vh.data(), m->d_val, (size_t)nnz * 4, hipMemcpyDeviceToHost);
            return ev == hipSuccess ? SM_OK : hip_fail(ev, "copy CSR values for the layout builder");
        };
        hipError_t e3 = hipSuccess;
        if (nnz) e3 = hipMemcpy(ch.data(), m->d_col, (size_t)nnz * 4, hipMemcpyDeviceToHost);
        st = e3 == hipSuccess ? SM_OK : hip_fail(e3, "copy CSR columns for the layout builder");
        if (st == SM_OK && xband) st = values();
        if (st == SM_OK && xband) st = upload_xband(m.get(), rp.data(), ch.data(), vh.data(), xband_kind_setting(m.get()));
        if (st == SM_OK && want_sweep(m.get())) st = values();
        if (st == SM_OK && want_sweep(m.get())) st = upload_sweep(m.get(), rp.data(), ch.data(), vh.data());
        if (st == SM_OK && want_relabel_size(m.get())) st = upload_relabel(m.get(), ch.data());
        if (st == SM_OK && want_ccsell(m.get())) st = values();
        if (st == SM_OK && want_ccsell(m.get())) st = upload_ccsell(m.get(), rp.data(), ch.data(), vh.data());
        if (st == SM_OK && want_sell(m.get())) st = values();
        if (st == SM_OK && want_sell(m.get())) st = upload_sell_layouts(m.get(), rp.data(), ch.data(), vh.data());
        if (st == SM_OK && want_merge_stage(m.get())) st = values();
        if (st == SM_OK && want_merge_stage(m.get()))
            st = upload_merge_stage(m.get(), rp.data(), ch.data(), vh.data());
    }
    if (st != SM_OK) { free_device(m.get()); return st; }
    *out = m.release();
    return SM_OK;
}

sm_status sm_get_info(const sm_matrix *m, sm_info *info) {
    return sm_get_info_ex(m, info, sizeof(sm_info));
}

sm_status sm_debug_seed_handoff(sm_matrix *m, uint64_t started) {
    if (!m) return fail(SM_ERR_INVALID_ARG, "null matrix");
    const XbandDev &xb = m->plan.xb;
    if (xb.n_blocks <= 0 || (xb.kind != kXbBand2 && xb.kind != kXbCband) || xb.n_slabs < 2 || !xb.d_tickets)
        return fail(SM_ERR_NOT_SUPPORTED, "no multi-slab band2/cband layout");
    if (started % (uint64_t)xb.n_slabs != 0)
        return fail(SM_ERR_NOT_SUPPORTED, "started must be a multiple of the slab count");
    DeviceGuard g(m->device);
    // Control words per block (xband_dev.h slab_handoff_epoch): [0..1] started, [2..3] arrive.
    std::vector<int32_t> h((size_t)xb.n_blocks * 4, 0);
    for (int32_t b = 0; b < xb.n_blocks; ++b) memcpy(&h[(size_t)b * 4], &started, 8);
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(xb.d_tickets, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    return e == hipSuccess ? SM_OK : hip_fail(e, "sm_debug_seed_handoff");
}

sm_status sm_get_info_ex(const sm_matrix *m, sm_info *out, size_t info_bytes) {
    if (!m || !out) return fail(SM_ERR_INVALID_ARG, "null argument");
    sm_info full;
    memset(&full, 0, sizeof(full));
    sm_info *info = &full;
    info->s_rows = m->s_rows;
    info->s_cols = m->s_cols;
    info->n_rows = m->n_rows;
    info->n_cols = m->n_cols;
    info->nnz = m->nnz;
    info->table_size = m->table_size;
    info->has_ref_stream = m->has_ref ? 1 : 0;
    info->n_entries = (int64_t)m->pos.size();
    info->n_panels = (int64_t)m->panel_col_off.size();
    info->device = m->device;
    info->n_tiles = m->plan.n_tiles;
    info->n_long_rows = m->plan.n_long;
    info->max_row_nnz = m->plan.max_row_nnz;
    info->has_xband = m->plan.xb.n_blocks > 0 ? m->plan.xb.kind : 0;
    info->xband_blocks = m->plan.xb.n_blocks;
    info->xband_bands = m->plan.xb.n_bands;
    info->xband_slabs = m->plan.xb.n_blocks > 0 ? m->plan.xb.n_slabs : 0;
    info->xband_block_rows = m->plan.xb.block_rows;
    info->xband_slab_cols =
        m->plan.xb.n_blocks == 0 ? 0
        : m->plan.xb.kind == kXbBand2 || m->plan.xb.kind == kXbCband || m->plan.xb.kind == kXbGcb
            ? m->plan.xb.slab_bands   // band2 / cband / gcb keep slab columns there
        : (int32_t)std::min<int64_t>((int64_t)m->plan.xb.slab_bands * m->plan.xb.band_cols, INT32_MAX);
    info->xband_slab0_cols = m->plan.xb.slab0_cols > 0 ? m->plan.xb.slab0_cols : info->xband_slab_cols;
    info->merge_stage = m->plan.d_mstage_w ? 1 : 0;
    info->xband_beta_last = SM_B2_BL && m->plan.xb.n_blocks > 0 && m->plan.xb.n_slabs > 1 &&
                            (m->plan.xb.kind == kXbBand2 || m->plan.xb.kind == kXbCband);
    info->device_bytes = m->device_bytes;
    info->col_relabel = m->plan.n_relabel > 0 ? 1 : 0;
    info->sell_slices = m->plan.sell.n_slices;
    info->sell_codebook = m->plan.sell.d_table != nullptr || m->plan.cc.d_table != nullptr;
    info->ccsell_chunks = m->plan.cc.n_slices > 0 ? m->plan.cc.n_chunks : 0;
    info->hot_cols = m->plan.hot.n_blocks > 0 ? m->plan.hot_cols : 0;
    info->sweep_blocks = (int32_t)std::min<int64_t>(m->plan.sw.n_blocks, INT32_MAX);
    info->exact_sell_slices = m->plan.xsell.n_slices;
    {
        const int a = exact_algo(m, true);
        info->exact_algo = a == kAlgoExactSell ? (int32_t)SM_ALGO_SELL : a;
    }
    // Only the bytes the caller's struct has (an older, shorter sm_info stays valid).
    memcpy(out, &full, std::min(info_bytes, sizeof(full)));
    return SM_OK;
}

sm_status sm_layout_digest(const sm_matrix *m, uint64_t digest[4]) {
    if (!m || !digest) return fail(SM_ERR_INVALID_ARG, "null argument");
    DeviceGuard g(m->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    for (int k = 0; k < 4; k++) digest[k] = 0;
    const Plan &p = m->plan;
    sm_status st = SM_OK;
    if (p.n_relabel > 0) {
        Fnv f;
        if ((st = fnv_dev(f, p.d_perm, p.n_relabel)) != SM_OK) return st;
        if ((st = fnv_dev(f, p.d_rcol, m->nnz)) != SM_OK) return st;
        digest[0] = f.h;
    }
    const XbandDev &xb = p.xb;
    if (xb.kind == kXbGcb && xb.n_blocks > 0) {   // gathered chunk bands (gcb.h)
        const int64_t ntile = (int64_t)xb.n_blocks * xb.n_slabs;
        Fnv f;
        const int32_t geo[5] = {xb.block_rows, xb.band_cols, xb.n_blocks, xb.n_slabs, xb.slab_bands};
        f.add(geo, sizeof(geo));
        if ((st = fnv_dev(f, xb.d_chunk_start, ntile + 1)) != SM_OK) return st;
        if ((st = fnv_dev(f, xb.d_band_clo, xb.n_bands)) != SM_OK) return st;
        digest[1] = f.h;
        Fnv w;
        if ((st = fnv_dev(w, xb.d_word, (int64_t)xb.n_bands * kGcbBandWords)) != SM_OK) return st;
        digest[2] = w.h;
    }
    const SellDev &d = p.sell;
    if (d.n_slices > 0) {
        std::vector<int64_t> off((size_t)d.n_slices);
        std::vector<int32_t> len((size_t)d.n_slices);
        SM_TRY_HIP(hipMemcpy(off.data(), d.d_off, off.size() * 8, hipMemcpyDeviceToHost));
        SM_TRY_HIP(hipMemcpy(len.data(), d.d_len, len.size() * 4, hipMemcpyDeviceToHost));
        const int64_t padded = off.back() + (int64_t)len.back() * kSellLanes;
        Fnv f;
        f.add(off.data(), off.size() * 8);
        f.add(len.data(), len.size() * 4);
        if ((st = fnv_dev(f, d.d_row, d.n_slices * kSellLanes)) != SM_OK) return st;
        if ((st = fnv_dev(f, d.d_row_len, d.n_slices * kSellLanes)) != SM_OK) return st;
        f.add(&d.n_long, 4);
        f.add(&d.max_len, 4);
        if ((st = fnv_dev(f, d.d_long_rows, d.n_long)) != SM_OK) return st;
        if ((st = fnv_dev(f, d.d_long_ptr, d.n_long > 0 ? d.n_long + 1 : 0)) != SM_OK) return st;
        digest[1] = f.h;
        Fnv c;
        if ((st = fnv_dev(c, d.d_col, padded + 32 * kSellLanes)) != SM_OK) return st;
        if ((st = fnv_dev(c, d.d_val, d.d_val ? padded + 32 * kSellLanes : 0)) != SM_OK) return st;
        digest[2] = c.h;
    }
    Fnv t;   // [3]: the sliced ELL's codebook, then the merge staging copy
    bool any = false;
    if (d.n_slices > 0 && d.d_table) {
        if ((st = fnv_dev(t, d.d_table, d.table_size)) != SM_OK) return st;
        t.add(&d.table_size, 4);
        any = true;
    }
    if (p.d_mstage_w) {
        if ((st = fnv_dev(t, p.d_mstage_w, m->nnz)) != SM_OK) return st;
        if ((st = fnv_dev(t, p.d_mstage_z, m->nnz)) != SM_OK) return st;
        if ((st = fnv_dev(t, p.d_mstage_tab, 256)) != SM_OK) return st;
        any = true;
    }
    if (any) digest[3] = t.h;
    return SM_OK;
}

int32_t sm_num_rows(const sm_matrix *m) { return m ? (int32_t)m->s_rows : 0; }
int32_t sm_num_cols(const sm_matrix *m) { return m ? (int32_t)m->s_cols : 0; }

sm_status sm_copy_ref_stream(const sm_matrix *m, uint8_t *pos, uint8_t *val, int32_t *pro,
                             int32_t *pco, int64_t *pb, int64_t *pe) {
    if (!m) return fail(SM_ERR_INVALID_ARG, "null matrix");
    if (!m->has_ref) return fail(SM_ERR_NOT_SUPPORTED, "matrix holds no reference encoding");
    if (pos && !m->pos.empty()) memcpy(pos, m->pos.data(), m->pos.size());
    if (val && !m->val.empty()) memcpy(val, m->val.data(), m->val.size());
    const size_t P = m->panel_col_off.size();
    if (pro && P) memcpy(pro, m->panel_row_off.data(), P * 4);
    if (pco && P) memcpy(pco, m->panel_col_off.data(), P * 4);
    if (pb && P) memcpy(pb, m->panel_begin.data(), P * 8);
    if (pe && P) memcpy(pe, m->panel_end.data(), P * 8);
    return SM_OK;
}

sm_status sm_build_ref_stream(sm_matrix *m, const float *table, int32_t table_size) {
    if (!m) return fail(SM_ERR_INVALID_ARG, "null matrix");
    if (m->has_ref) return SM_OK;
    if (table && (table_size < 0 || table_size > 255))
        return fail(SM_ERR_INVALID_ARG, "table_size %d not in [0, 255]", table_size);
    DeviceGuard g(m->device);
    // On the device (refenc_dev.hip): sort, gaps, scan and emit; the host keeps the stream's
    // copy (sm_copy_ref_stream, sm_equal) and derives the native layout's batch metadata.
    EncodeResult er;
    hipError_t he = hipSuccess;
    const int rc = encode_csr_ref_device(m->d_row_ptr, m->d_col, m->d_val, nullptr, m->n_rows, m->n_cols,
                                         m->nnz, table, table_size, er, nullptr, he);
    if (rc == -5) return hip_fail(he, "sm_build_ref_stream");
    if (rc == -2) return fail(SM_ERR_INVALID_ARG, "a value is not in the codebook");
    if (rc == -3) return fail(SM_ERR_NOT_SUPPORTED, "more than 255 distinct values: no uint8 ids");
    if (rc == -4) return fail(SM_ERR_NOT_SUPPORTED, "S rows >= 2^23: the reference's int32 offsets overflow");
    if (rc != 0) return fail(SM_ERR_INVALID_ARG, "bad codebook");
    m->table_size = er.table_size;
    m->table = std::move(er.table);
    m->pos = std::move(er.pos);
    m->val = std::move(er.val_id);
    m->panel_row_off = std::move(er.panel_row_off);
    m->panel_col_off = std::move(er.panel_col_off);
    m->panel_begin = std::move(er.panel_begin);
    m->panel_end = std::move(er.panel_end);
    m->has_ref = true;
    const sm_status st = upload_native(m);
    if (st != SM_OK) {   // no half-built encoding -- a retry starts over
        free_native_dev(m->plan.nat);
        m->has_ref = false;
        m->table_size = 0;
        for (auto *v : {&m->pos, &m->val}) std::vector<uint8_t>().swap(*v);
        std::vector<float>().swap(m->table);
        std::vector<int32_t>().swap(m->panel_row_off);
        std::vector<int32_t>().swap(m->panel_col_off);
        std::vector<int64_t>().swap(m->panel_begin);
        std::vector<int64_t>().swap(m->panel_end);
    }
    return st;
}

sm_status sm_copy_csr(const sm_matrix *m, int32_t *row_ptr, int32_t *col_idx, float *val) {
    if (!m) return fail(SM_ERR_INVALID_ARG, "null matrix");
    DeviceGuard g(m->device);
    if (row_ptr)
        SM_TRY_HIP(hipMemcpy(row_ptr, m->d_row_ptr, (size_t)(m->n_rows + 1) * 4, hipMemcpyDeviceToHost));
    if (col_idx && m->nnz)
        SM_TRY_HIP(hipMemcpy(col_idx, m->d_col, (size_t)m->nnz * 4, hipMemcpyDeviceToHost));
    if (val && m->nnz)
        SM_TRY_HIP(hipMemcpy(val, m->d_val, (size_t)m->nnz * 4, hipMemcpyDeviceToHost));
    return SM_OK;
}

sm_status sm_to_dense(const sm_matrix *m, float *out, int32_t stride, sm_trans trans) {
    if (!m) return fail(SM_ERR_INVALID_ARG, "null matrix");
    if (trans != SM_NO_TRANS && trans != SM_TRANS) return fail(SM_ERR_INVALID_ARG, "bad trans");
    // NoTrans: S, s_rows x stride (s_cols used); Trans: S^T = B, s_cols x stride (s_rows used)
    const int64_t out_rows = trans == SM_TRANS ? m->s_cols : m->s_rows;
    const int64_t width = trans == SM_TRANS ? m->s_rows : m->s_cols;
    if (out_rows == 0) return SM_OK;
    if (!out || stride < width) return fail(SM_ERR_INVALID_ARG, "null out or stride < %lld", (long long)width);
    DeviceGuard g(m->device);
    const size_t bytes = (size_t)out_rows * stride * sizeof(float);
    float *d = nullptr;
    SM_TRY_HIP(hipMalloc((void **)&d, bytes));
    hipError_t e = hipMemsetAsync(d, 0, bytes, 0);
    if (e == hipSuccess)
        e = launch_scatter_dense((int32_t)m->n_rows, m->d_row_ptr, m->d_col, m->d_val, d, stride,
                                 trans == SM_TRANS, 0);
    if (e == hipSuccess) e = hipMemcpy(out, d, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return hip_fail(e, "sm_to_dense");
    return SM_OK;
}

int32_t sm_equal(const sm_matrix *a, const sm_matrix *b) {
    if (!a || !b) return 0;
    if (a == b) return 1;
    if (a->s_rows != b->s_rows || a->s_cols != b->s_cols || a->nnz != b->nnz) return 0;
    if (a->has_ref && b->has_ref) {
        // the reference's own member-wise comparison (sparse-matrix.cc:197-207)
        if (a->table.size() != b->table.size() ||
            memcmp(a->table.data(), b->table.data(), a->table.size() * 4) != 0)
            return 0;
        return a->pos == b->pos && a->val == b->val && a->panel_row_off == b->panel_row_off &&
               a->panel_col_off == b->panel_col_off && a->panel_begin == b->panel_begin &&
               a->panel_end == b->panel_end;
    }
    std::vector<int32_t> ra((size_t)a->n_rows + 1), rb((size_t)b->n_rows + 1);
    std::vector<int32_t> ca((size_t)a->nnz), cb((size_t)b->nnz);
    std::vector<float> va((size_t)a->nnz), vb((size_t)b->nnz);
    if (sm_copy_csr(a, ra.data(), ca.data(), va.data()) != SM_OK) return 0;
    if (sm_copy_csr(b, rb.data(), cb.data(), vb.data()) != SM_OK) return 0;
    return ra == rb && ca == cb &&
           (va.empty() || memcmp(va.data(), vb.data(), va.size() * 4) == 0);
}

// ---------------------------------------------------------------------------

sm_status sm_spmv(const sm_matrix *m, float alpha, const float *x, float beta, float *y,
                  sm_algo algo, sm_stream stream) {
    if (!m) return fail(SM_ERR_INVALID_ARG, "null matrix");
    if (m->n_rows == 0) return SM_OK;
    if (!y || (alpha != 0.0f && m->n_cols > 0 && !x)) return fail(SM_ERR_INVALID_ARG, "null x/y");
    DeviceGuard g(m->device);
    hipStream_t s = (hipStream_t)stream;
    const int32_t n = (int32_t)m->n_rows;
    hipError_t e = hipSuccess;
    if (alpha == 0.0f) {   // sparse-matrix.cc:149-152: only the beta pass
        if (beta != 1.0f) e = launch_beta(y, 1, n, n, beta, s);
        return e == hipSuccess ? SM_OK : hip_fail(e, "sm_spmv beta");
    }
    if (algo == SM_ALGO_NATIVE) {   // the reference stream: y = x * S (a = x, c = y, m = 1)
        if (!m->has_ref || (m->plan.nat.n_panels == 0 && m->nnz > 0))
            return fail(SM_ERR_NOT_SUPPORTED, "SM_ALGO_NATIVE needs a matrix built from the dense index");
        e = m->plan.nat.n_panels == 0
                ? (beta != 1.0f ? launch_beta(y, 1, n, n, beta, s) : hipSuccess)
                : with_scratch(m, s, native_scratch(m->plan.nat), [&] {
                      return launch_native_addmatmat(m->plan.nat, 1, x, (int32_t)m->n_cols, y, n, alpha,
                                                     beta, s);
                  });
        e = after_launch(e, s, "sm_spmv native");
        return e == hipSuccess ? SM_OK : hip_fail(e, "sm_spmv native");
    }
    if (algo == SM_ALGO_MFMA) return fail(SM_ERR_NOT_SUPPORTED, "SM_ALGO_MFMA is an SpMM algorithm (n_rhs = 32)");
    const int ai = algo == SM_ALGO_EXACT ? exact_algo(m, ((uintptr_t)x % 16) == 0) : (int)algo;
    if ((ai < SM_ALGO_AUTO || ai > SM_ALGO_SELL) && ai != kAlgoExactSell && ai != SM_ALGO_MERGE)
        return fail(SM_ERR_INVALID_ARG, "unknown algo %d", (int)algo);
    // The matrix's SpMV scratch (sm_internal.h): SpMVs that use it run one after the
    // other on the device, whatever stream or thread issues them.
    const Plan &pl = m->plan;
    const bool scratch = ai == SM_ALGO_MERGE ||
                         (ai != SM_ALGO_PARITY && ai != SM_ALGO_VECTOR &&
                          ((pl.xb.n_blocks > 0 && pl.xb.n_slabs > 1) || pl.n_relabel > 0 ||
                           (pl.hot.n_blocks > 0 && pl.hot.n_slabs > 1) ||
                           pl.sell.n_long > 0 || pl.n_long > 0));
    std::unique_lock<std::mutex> lk(m->scratch_mu, std::defer_lock);
    bool ordered = false;
    if (scratch) {
        lk.lock();
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cs) != hipSuccess) cs = hipStreamCaptureStatusNone;
        ordered = cs == hipStreamCaptureStatusNone;
        if (ordered && !m->scratch_ready)
            e = hipEventCreateWithFlags(&m->scratch_ready, hipEventDisableTiming);
        if (ordered && e == hipSuccess && m->scratch_recorded) e = hipStreamWaitEvent(s, m->scratch_ready, 0);
        if (e != hipSuccess) return hip_fail(e, "sm_spmv scratch ordering");
    }
    switch (ai) {
    case SM_ALGO_PARITY:
        e = launch_spmv_parity(n, m->d_row_ptr, m->d_col, m->d_val, x, y, alpha, beta, s);
        break;
    case SM_ALGO_VECTOR:
        e = launch_spmv_vector(n, m->plan.avg_row_nnz, m->d_row_ptr, m->d_col, m->d_val, x, y,
                               alpha, beta, s);
        break;
    case SM_ALGO_AUTO:
    case SM_ALGO_XBAND:
        if (m->plan.sw.n_blocks > 0) {   // column-swept row blocks: no scratch, bit-identical
            e = launch_spmv_sweep(m->plan.sw, n, (int32_t)m->n_cols, x, y, alpha, beta, s);
            break;
        }
        if (m->plan.xb.n_blocks > 0 && ((uintptr_t)x % 16) == 0) {
            e = m->plan.xb.kind == kXbBand2 || m->plan.xb.kind == kXbCband
                    ? launch_spmv_band2(m->plan.xb, n, (int32_t)m->n_cols, x, y, alpha, beta, s)
                : m->plan.xb.kind == kXbGcb
                    ? launch_spmv_gcb(m->plan.xb, n, (int32_t)m->n_cols, x, y, alpha, beta, s)
                    : launch_spmv_xband(m->plan.xb, n, (int32_t)m->n_cols, x, y, alpha, beta, s);
            break;
        }
        // fall through: no band layout (or unaligned x) -> sell or stream kernel
        [[fallthrough]];
    case SM_ALGO_SELL:
        if (m->plan.cc.n_slices > 0) {   // column-chunked: no scratch, y read and written per chunk
            e = launch_spmv_ccsell(m->plan.cc, x, y, alpha, beta, s);
            break;
        }
        if (m->plan.sell.n_slices > 0) {
            const float *xs = x;
            if (m->plan.n_relabel > 0) {   // the slices hold relabeled columns
                e = launch_x_relabel(m->plan.n_relabel, m->plan.d_perm, x, m->plan.d_xperm, s);
                xs = m->plan.d_xperm;
            }
            float b = beta;
            if (e == hipSuccess && m->plan.hot.n_blocks > 0) {   // hot columns first, then the rest
                e = launch_spmv_band2(m->plan.hot, n, m->plan.hot_cols, xs, y, alpha, beta, s);
                b = 1.0f;
            }
            if (e == hipSuccess) e = launch_spmv_sell(m->plan.sell, xs, y, alpha, b, s);
            break;
        }
        [[fallthrough]];   // no sell layout -> stream kernel
    case SM_ALGO_STREAM:
        // Long-row partial sums (and the relabeled x) live in the matrix (allocated at
        // creation): SpMVs on one matrix must not run concurrently on different streams.
        if (m->plan.n_relabel > 0) {
            e = launch_x_relabel(m->plan.n_relabel, m->plan.d_perm, x, m->plan.d_xperm, s);
            if (e == hipSuccess)
                e = launch_spmv_stream(m->plan, m->d_row_ptr, m->plan.d_rcol, m->d_val,
                                       m->plan.d_xperm, y, alpha, beta, m->plan.d_partials, s);
            break;
        }
        e = launch_spmv_stream(m->plan, m->d_row_ptr, m->d_col, m->d_val, x, y, alpha, beta,
                               m->plan.d_partials, s);
        break;
    case SM_ALGO_MERGE: {   // merge path over the CSR arrays (kernels_merge.hip)
        const MergeStage mstage{m->plan.d_mstage_w, m->plan.d_mstage_z, m->plan.d_mstage_tab};
        if (m->plan.n_relabel > 0) {   // skewed columns: the relabeled copy, hot x in L2 (as stream)
            e = launch_x_relabel(m->plan.n_relabel, m->plan.d_perm, x, m->plan.d_xperm, s);
            if (e == hipSuccess)
                e = launch_spmv_merge(n, (int32_t)m->nnz, m->d_row_ptr, m->plan.d_rcol, m->d_val, m->plan.d_xperm, y,
                                      alpha, beta, m->plan.d_merge_corner, m->plan.d_merge, s, &mstage);
            break;
        }
        e = launch_spmv_merge(n, (int32_t)m->nnz, m->d_row_ptr, m->d_col, m->d_val, x, y, alpha, beta,
                              m->plan.d_merge_corner, m->plan.d_merge, s, &mstage);
        break;
    }
    case kAlgoExactSell: {   // unsegmented slices: every row in stored order, one lane each
        const float *xs = x;
        if (m->plan.n_relabel > 0) {   // the slices hold relabeled columns
            e = launch_x_relabel(m->plan.n_relabel, m->plan.d_perm, x, m->plan.d_xperm, s);
            xs = m->plan.d_xperm;
        }
        if (e == hipSuccess) e = launch_spmv_sell(m->plan.xsell, xs, y, alpha, beta, s);
        break;
    }
    default:
        return fail(SM_ERR_INVALID_ARG, "unknown algo %d", (int)algo);
    }
    if (ordered) {   // whatever was queued (also on a failed launch) uses the scratch
        const hipError_t er = hipEventRecord(m->scratch_ready, s);
        if (er == hipSuccess) m->scratch_recorded = true;
        if (e == hipSuccess) e = er;
    }
    e = after_launch(e, s, "sm_spmv");
    return e == hipSuccess ? SM_OK : hip_fail(e, "sm_spmv launch");
}

sm_status sm_spmm(const sm_matrix *m, int32_t n_rhs, float alpha, const float *X, int64_t ldx,
                  float beta, float *Y, int64_t ldy, sm_algo algo, sm_stream stream) {
    if (!m) return fail(SM_ERR_INVALID_ARG, "null matrix");
    if (n_rhs < 0) return fail(SM_ERR_INVALID_ARG, "n_rhs < 0");
    if (m->n_rows == 0 || n_rhs == 0) return SM_OK;
    if (ldy < n_rhs || ldx < n_rhs) return fail(SM_ERR_INVALID_ARG, "ldx/ldy < n_rhs");
    if (!Y || (alpha != 0.0f && m->n_cols > 0 && !X)) return fail(SM_ERR_INVALID_ARG, "null X/Y");
    DeviceGuard g(m->device);
    hipStream_t s = (hipStream_t)stream;
    const int32_t n = (int32_t)m->n_rows;
    hipError_t e;
    if (alpha == 0.0f) {
        e = beta != 1.0f ? launch_beta(Y, n, n_rhs, ldy, beta, s) : hipSuccess;
        return e == hipSuccess ? SM_OK : hip_fail(e, "sm_spmm beta");
    }
    if (algo == SM_ALGO_MFMA) {   // the matrix-core SpMM (spmm_mfma.hip)
        if (n_rhs != 32 || ldx % 2 || ldy % 2 || ((uintptr_t)X % 8) || ((uintptr_t)Y % 8) ||
            (uint64_t)m->n_cols * (uint64_t)ldx * 4u >= 0xFFFFFFF0ull)
            return fail(SM_ERR_NOT_SUPPORTED, "SM_ALGO_MFMA needs n_rhs = 32, even ldx/ldy, 8-byte "
                        "aligned X/Y and X under 4 GiB");
        e = launch_spmm_mfma(n, m->d_row_ptr, m->d_col, m->d_val, (int32_t)m->nnz, X, ldx, m->n_cols,
                             Y, ldy, alpha, beta, s);
        e = after_launch(e, s, "sm_spmm mfma");
        return e == hipSuccess ? SM_OK : hip_fail(e, "sm_spmm mfma");
    }
    const bool vec_ok = n_rhs % 4 == 0 && n_rhs <= 128 && ldx % 4 == 0 && ldy % 4 == 0 &&
                        ((uintptr_t)X % 16) == 0 && ((uintptr_t)Y % 16) == 0;
    if (algo == SM_ALGO_SELL || algo == SM_ALGO_XBAND || algo == SM_ALGO_EXACT || algo == SM_ALGO_MERGE)
        algo = SM_ALGO_AUTO;   // SpMV layouts; the SpMM kernels keep every row's order
    if ((algo == SM_ALGO_AUTO || algo == SM_ALGO_STREAM || algo == SM_ALGO_VECTOR) && vec_ok)
        e = launch_spmm_rowpanel(n, n_rhs, m->d_row_ptr, m->d_col, m->d_val, (int32_t)m->nnz, X,
                                 ldx, m->n_cols, Y, ldy, alpha, beta, algo != SM_ALGO_VECTOR, s);
    else if (algo >= SM_ALGO_AUTO && algo <= SM_ALGO_VECTOR)
        e = launch_spmm_generic(n, n_rhs, m->d_row_ptr, m->d_col, m->d_val, X, ldx, 1, Y, ldy, 1,
                                alpha, beta, true, s);
    else
        return fail(SM_ERR_INVALID_ARG, "unknown algo %d", (int)algo);
    e = after_launch(e, s, "sm_spmm");
    return e == hipSuccess ? SM_OK : hip_fail(e, "sm_spmm launch");
}

sm_status sm_addmatmat(const sm_matrix *mat, const float *a, int32_t m, int32_t lda, float *c,
                       int32_t ldc, float alpha, float beta, sm_algo algo, sm_stream stream) {
    if (!mat) return fail(SM_ERR_INVALID_ARG, "null matrix");
    const int64_t k = mat->s_rows, n = mat->s_cols;
    if (m < 0) return fail(SM_ERR_INVALID_ARG, "m < 0");
    if (m == 0 || n == 0) return SM_OK;
    if (ldc < n || (alpha != 0.0f && lda < k)) return fail(SM_ERR_INVALID_ARG, "lda/ldc too small");
    if (!c || (alpha != 0.0f && k > 0 && !a)) return fail(SM_ERR_INVALID_ARG, "null a/c");
    if (m == 1 && algo != SM_ALGO_NATIVE) return sm_spmv(mat, alpha, a, beta, c, algo, stream);
    DeviceGuard g(mat->device);
    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    if (alpha == 0.0f) {
        e = beta != 1.0f ? launch_beta(c, m, (int32_t)n, ldc, beta, s) : hipSuccess;
        return e == hipSuccess ? SM_OK : hip_fail(e, "sm_addmatmat beta");
    }
    if (algo == SM_ALGO_NATIVE) {   // the reference stream, A and C read in place
        if (!mat->has_ref || (mat->plan.nat.n_panels == 0 && mat->nnz > 0))
            return fail(SM_ERR_NOT_SUPPORTED, "SM_ALGO_NATIVE needs a matrix built from the dense index");
        e = mat->plan.nat.n_panels == 0
                ? (beta != 1.0f ? launch_beta(c, m, (int32_t)n, ldc, beta, s) : hipSuccess)
                : with_scratch(mat, s, native_scratch(mat->plan.nat), [&] {
                      return launch_native_addmatmat(mat->plan.nat, m, a, lda, c, ldc, alpha, beta, s);
                  });
        e = after_launch(e, s, "sm_addmatmat native");
        return e == hipSuccess ? SM_OK : hip_fail(e, "sm_addmatmat native");
    }
    // Few right-hand sides on a matrix of few B rows: the row-panel kernel gives each B row
    // mp / 4 lanes, so at m <= 4 and n = 16384 it runs 16384 lanes, each a serial chain over
    // its whole row.  Two remedies, both keeping every output's terms in stored order:
    //  - short rows (<= 64 terms on average) and m <= 2: m SpMVs on A's and C's rows (x = A
    //    row i, y = C row i, contiguous, no transposes), each with a reference-order kernel
    //    (EXACT) so the result equals the row panel's bit for bit whatever m is;
    //  - otherwise the row panel on a workspace padded to 16 columns (4 lanes per B row; the
    //    padding columns are computed and never copied back).
    // blas_test 16384^2 at 25 % (rows of ~4096 terms), AUTO, round 4: m = 4 0.957 ms as four
    // SpMVs, m = 16 0.425 ms (profiles/r04_blas_test_16384_fewrhs.txt).
    const bool few_rows = n < ((int64_t)1 << 18) && k > 0 && algo != SM_ALGO_PARITY;
    if (few_rows && m <= 2 && mat->nnz <= 64 * n) {
        const sm_algo sa = (algo == SM_ALGO_AUTO || algo == SM_ALGO_EXACT) ? SM_ALGO_EXACT : algo;
        for (int32_t i = 0; i < m; i++) {
            const sm_status st = sm_spmv(mat, alpha, a + (int64_t)i * lda, beta, c + (int64_t)i * ldc, sa, stream);
            if (st != SM_OK) return st;
        }
        return SM_OK;
    }
    if (algo != SM_ALGO_PARITY && m > 128 && k > 0) {
        // Rows of A and C are independent products: row-panel calls of <= 128 rows each.
        for (int32_t i0 = 0; i0 < m; i0 += 128) {
            const sm_status st = sm_addmatmat(mat, a + (int64_t)i0 * lda, std::min<int32_t>(128, m - i0),
                                              lda, c + (int64_t)i0 * ldc, ldc, alpha, beta, algo, stream);
            if (st != SM_OK) return st;
        }
        return SM_OK;
    }
    if (algo != SM_ALGO_PARITY && m <= 128 && k > 0) {
        // C^T = B A^T through the row-panel SpMM (the reference transposes too,
        // kernel.cc:31-187): X = A^T (k x mp), Y = C^T (n x mp) in a stream-ordered
        // workspace, mp = m rounded up to 4 (the padding columns are never copied
        // back), then C = Y^T.  Same terms in the same order as the in-place kernel
        // below (bit-identical); the matrix is streamed once instead of m times.
        const int64_t mp = few_rows && m < 16 ? 16 : (m + 3) & ~3;
        // The matrix's workspace (sm_internal.h), where the reference allocates a temp
        // buffer per call (sparse-matrix.cc:155-161): stream-ordered behind the previous
        // call's kernels, so back-to-back calls neither block the host nor share bytes.
        const size_t ws_bytes = (size_t)(k + n) * mp * sizeof(float);
        std::lock_guard<std::mutex> lk(mat->ws_mu);
        e = hipSuccess;
        if (!mat->ws_ready) e = hipEventCreateWithFlags(&mat->ws_ready, hipEventDisableTiming);
        else e = hipStreamWaitEvent(s, mat->ws_ready, 0);
        if (e == hipSuccess && mat->ws_bytes < ws_bytes) {
            // Grow: the old buffer is released once its last user has finished.
            e = hipEventSynchronize(mat->ws_ready);
            if (e == hipSuccess) e = hipFree(mat->d_ws);
            mat->d_ws = nullptr;
            mat->ws_bytes = 0;
            if (e == hipSuccess) e = hipMalloc((void **)&mat->d_ws, ws_bytes);
            if (e == hipSuccess) mat->ws_bytes = ws_bytes;
            else mat->d_ws = nullptr;
        }
        float *X = mat->d_ws, *Y = mat->d_ws + k * mp;
        bool queued = false;   // any kernel on the workspace: the next user must wait for it
        if (e == hipSuccess) e = launch_transpose(a, m, (int32_t)k, lda, X, mp, s);
        queued = queued || e == hipSuccess;
        if (e == hipSuccess) e = launch_transpose(c, m, (int32_t)n, ldc, Y, mp, s);
        if (e == hipSuccess)
            e = launch_spmm_rowpanel((int32_t)n, mp == 16 && m < 16 ? 16 : m, mat->d_row_ptr, mat->d_col,
                                     mat->d_val, (int32_t)mat->nnz, X, mp, k, Y, mp, alpha, beta, true, s);
        if (e == hipSuccess) e = launch_transpose(Y, (int32_t)n, m, mp, c, ldc, s);
        if (queued) {   // recorded on the error path too: kernels may be queued
            const hipError_t er = hipEventRecord(mat->ws_ready, s);
            if (e == hipSuccess) e = er;
        }
        e = after_launch(e, s, "sm_addmatmat");
        return e == hipSuccess ? SM_OK : hip_fail(e, "sm_addmatmat (row panels)");
    }
    // Parity (or m > 128): C^T = B A^T read in place, one thread per output:
    // X(kk, i) = a[i*lda + kk], Y(j, i) = c[i*ldc + j].
    e = launch_spmm_generic((int32_t)n, m, mat->d_row_ptr, mat->d_col, mat->d_val, a, 1, lda, c,
                            1, ldc, alpha, beta, false, s);
    e = after_launch(e, s, "sm_addmatmat");
    return e == hipSuccess ? SM_OK : hip_fail(e, "sm_addmatmat launch");
}

sm_status sm_addmatmat_host(const sm_matrix *mat, const float *a, int32_t m, int32_t lda, float *c,
                            int32_t ldc, float alpha, float beta) {
    if (!mat) return fail(SM_ERR_INVALID_ARG, "null matrix");
    const int64_t k = mat->s_rows, n = mat->s_cols;
    if (m < 0) return fail(SM_ERR_INVALID_ARG, "m < 0");
    if (m == 0 || n == 0) return SM_OK;
    if (ldc < n || (alpha != 0.0f && lda < k)) return fail(SM_ERR_INVALID_ARG, "lda/ldc too small");
    if (!c || (alpha != 0.0f && k > 0 && !a)) return fail(SM_ERR_INVALID_ARG, "null a/c");
    DeviceGuard g(mat->device);
    const int64_t a_elems = (alpha != 0.0f && k > 0) ? (int64_t)(m - 1) * lda + k : 0;
    const int64_t c_elems = (int64_t)(m - 1) * ldc + n;
    float *da = nullptr, *dc = nullptr;
    hipError_t e = hipSuccess;
    if (a_elems) e = hipMalloc((void **)&da, (size_t)a_elems * 4);
    if (e == hipSuccess) e = hipMalloc((void **)&dc, (size_t)c_elems * 4);
    if (e == hipSuccess && a_elems) e = hipMemcpy(da, a, (size_t)a_elems * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dc, c, (size_t)c_elems * 4, hipMemcpyHostToDevice);
    sm_status st = SM_OK;
    if (e == hipSuccess) {
        // Bit-exact: the fastest reference-order kernels (SM_ALGO_EXACT: m = 1 a
        // reference-order SpMV layout, else parity; m > 1 the row-panel path).
        st = sm_addmatmat(mat, da, m, lda, dc, ldc, alpha, beta, SM_ALGO_EXACT, nullptr);
        if (st == SM_OK) e = hipMemcpy(c, dc, (size_t)c_elems * 4, hipMemcpyDeviceToHost);
    }
    (void)hipFree(da);
    (void)hipFree(dc);
    if (st != SM_OK) return st;
    return e == hipSuccess ? SM_OK : hip_fail(e, "sm_addmatmat_host");
}

sm_status sm_beta_scale(float *c, int32_t m, int32_t n, int32_t ldc, float beta, sm_stream stream) {
    if (m < 0 || n < 0 || (m > 0 && ldc < n)) return fail(SM_ERR_INVALID_ARG, "bad shape");
    if ((int64_t)m * n == 0) return SM_OK;
    if (!c) return fail(SM_ERR_INVALID_ARG, "null c");
    hipError_t e = launch_beta(c, m, n, ldc, beta, (hipStream_t)stream);
    return e == hipSuccess ? SM_OK : hip_fail(e, "sm_beta_scale");
}

sm_status sm_transpose(const float *a, int32_t m, int32_t n, int32_t lda, float *sa, int32_t ldsa,
                       sm_stream stream) {
    if (m < 0 || n < 0 || (m > 0 && lda < n) || (n > 0 && ldsa < m))
        return fail(SM_ERR_INVALID_ARG, "bad shape");   // kernel.cc:33 asserts ldsa >= m
    if ((int64_t)m * n == 0) return SM_OK;
    if (!a || !sa) return fail(SM_ERR_INVALID_ARG, "null pointer");
    hipError_t e = launch_transpose(a, m, n, lda, sa, ldsa, (hipStream_t)stream);
    return e == hipSuccess ? SM_OK : hip_fail(e, "sm_transpose");
}

sm_status sm_panel_kernel(int32_t variant, int32_t m, int32_t n, int32_t k, const float *a,
                          int32_t lda, float *c, int32_t ldc, float alpha, const uint8_t *ppos,
                          const uint8_t *pval, int32_t pos_len, const float *table,
                          int32_t valid_table_size, sm_stream stream) {
    if (variant < 0 || variant > 3) return fail(SM_ERR_INVALID_ARG, "variant must be 0..3");
    if (m < 0 || n < 0 || k < 0 || n > 256 || pos_len < 0)
        return fail(SM_ERR_INVALID_ARG, "bad panel shape m=%d n=%d k=%d pos_len=%d", m, n, k, pos_len);
    if (valid_table_size < 0 || valid_table_size > 255)
        return fail(SM_ERR_INVALID_ARG, "valid_table_size not in [0, 255]");
    const bool tr = variant >= 2;
    if (m > 0 && ((!tr && (lda < k || ldc < n)) || (tr && (lda < m || ldc < m))))
        return fail(SM_ERR_INVALID_ARG, "lda/ldc too small for variant %d", variant);
    if ((int64_t)m * n == 0 || pos_len == 0) return SM_OK;
    if (!a || !c || !ppos || !pval || !table) return fail(SM_ERR_INVALID_ARG, "null pointer");
    hipStream_t s = (hipStream_t)stream;
    void *ws = nullptr;
    // Not a hot path: a plain allocation, synchronised before it is released.
    hipError_t e = hipMalloc(&ws, panel_kernel_workspace_bytes(pos_len, n));
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(panel workspace)");
    e = launch_panel_kernel(variant, m, n, k, a, lda, c, ldc, alpha, ppos, pval, pos_len, table,
                            valid_table_size, ws, s);
    hipError_t e2 = hipStreamSynchronize(s);
    if (e == hipSuccess) e = e2;
    (void)hipFree(ws);
    return e == hipSuccess ? SM_OK : hip_fail(e, "sm_panel_kernel");
}

sm_status sm_stream_sync(sm_stream stream) {
    hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    if (e == hipSuccess) e = hipGetLastError();
    return e == hipSuccess ? SM_OK : hip_fail(e, "sm_stream_sync");
}

}  // extern "C"
