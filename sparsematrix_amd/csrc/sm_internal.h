// sm_internal.h -- internal types shared by the C-ABI host code and the HIP
// kernels of libsparsematrix_amd.so.  Not installed; the public surface is
// include/sparsematrix.h.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "sparsematrix.h"
#include "merge.h"

namespace smamd {

// ---- stream-kernel geometry (see DESIGN.md "Kernels") ----------------------
constexpr int kStreamThreads = 256;       // 4 wavefronts per workgroup
constexpr int kTileNnz = 4096;            // default terms staged in LDS per row tile (16 KiB)
constexpr int kTileRows = 1024;           // row cap per tile (empty-row heavy graphs)
constexpr int kLongChunk = 4096;          // terms per workgroup for rows > kTileNnz
constexpr int kSerialRowMax = SM_SERIAL_ROW_MAX;  // rows summed in reference order
constexpr int kPadElems = 64;             // zero tail on col/val for aligned x4 loads

// Development knobs.  Builds with -DSM_DEV (tools/*_ab.sh) read SM_* environment
// variables for A/B measurements and ablations; the shipped library reads none of
// them (a stray variable cannot change a caller's layouts or results) and holds no
// ablation kernels.  Layout choices reach it only through sm_build_opts.
inline const char *dev_env(const char *name) {
#ifdef SM_DEV
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// Resolved layout options (sm_build_opts with defaults filled in).
struct BuildOpts {
    int32_t layout = SM_LAYOUT_AUTO;
    int32_t band_slabs = 0;
    int32_t band_tall = 0;
    int32_t gather_band_log2 = 0;
    int32_t sell = -1;
    int32_t sell_codebook = -1;
    int32_t sell_max_len = 0;
    int32_t sell_streams = 0;
    int64_t sell_sigma = 0;
    int32_t relabel = -1;
    int32_t tile_nnz = 0;
    int32_t ccsell = -1;
    int32_t ccsell_chunk_log2 = 0;
    int32_t hot_cols = 0;
    int32_t exact_sell = 0;   // 0 auto, 1 always, -1 never (sm_build_opts.exact_sell)
    int32_t band_slab0_permille = 0;   // 0 auto (sm_build_opts.band_slab0_permille)
    int32_t merge_stage = 0;           // sm_build_opts.merge_stage
    int32_t host_build = 0;            // sm_build_opts.host_build
};

// Row tile: rows [r0, r1) whose terms fit one LDS tile.  flags bit0: the tile
// holds a row longer than kSerialRowMax (wave-parallel reduction pass needed).
struct alignas(16) Tile {
    int32_t r0, r1, flags, pad;
};

// Chunk of a long row: terms [begin, end) of long row `lr` (index into
// long_rows).  Partial sums are combined in chunk order by the finalize kernel.
struct alignas(16) Chunk {
    int32_t lr, begin, end, pad;
};

// Device copy of the column-band layout (xband.h).
struct XbandDev {
    int32_t kind = 0;                 // XbKind; 0 when not built
    int32_t threads = 0;              // workgroup size of the kind
    int32_t block_rows = 0, band_cols = 0, n_blocks = 0, n_bands = 0;
    int32_t n_slabs = 1, slab_bands = 0;   // tiles = n_blocks * n_slabs
    int32_t slab0_cols = 0;           // band2 / cband: columns of slab 0 (others: slab_bands)
    int64_t n_chunks = 0;
    int64_t max_chunks_per_band = 0;
    int32_t *d_chunk_start = nullptr;
    uint32_t *d_word = nullptr;
    float *d_val = nullptr;
    float *d_partials = nullptr;      // (n_slabs - 1) * n_rows slab partial sums (one SpMV in flight)
    int32_t *d_tickets = nullptr;     // 4 x n_blocks slab hand-off control words, zero between SpMVs
    // band2 kind (band2.cpp): d_chunk_start = tile -> first band (n_tiles + 1), d_word =
    // the lane-interleaved entries (4096 per band), d_band_clo = each band's first column.
    int32_t *d_band_clo = nullptr;
    // cband kind: the codebook (table_size <= 255 floats) the entries' ids index.
    float *d_table = nullptr;
    int32_t table_size = 0;
    // gcb kind: column pacing words (kernels_gcb.hip), 8 x (1 + pace_k) monotonic counters.
    int32_t *d_pace = nullptr;
    int32_t pace_k = 0;
};

// Device copy of the sorted sliced-ELL layout (sell.h).
struct SellDev {
    int64_t n_slices = 0;             // 0 when not built
    int64_t *d_off = nullptr;         // n_slices
    int32_t *d_len = nullptr;         // n_slices
    int32_t *d_row = nullptr;         // n_slices * 64 (-1: no row)
    int32_t *d_row_len = nullptr;     // n_slices * 64
    int32_t *d_col = nullptr;         // padded slots (relabeled columns when n_relabel > 0)
    float *d_val = nullptr;           // nullptr in the codebook form
    // Codebook form (sell.h): d_col holds column | id << 24 words, values in d_table.
    float *d_table = nullptr;         // table_size fp32 values (nullptr: plain form)
    int32_t table_size = 0;
    int32_t max_len = 0;              // rows up to this length are whole lanes
    // Rows longer than max_len: cut in segments (lanes with row = -2 - partial).
    int32_t n_long = 0;
    int32_t *d_long_rows = nullptr;   // n_long
    int32_t *d_long_ptr = nullptr;    // n_long + 1 offsets into d_partials
    float *d_partials = nullptr;      // one per segment (one SpMV in flight per matrix)
};

// Device copy of the column-chunked sorted sliced-ELL layout (ccsell.h).
struct CcsellDev {
    int64_t n_slices = 0;             // 0 when not built
    int32_t n_chunks = 0, chunk_log2 = 0;
    std::vector<int64_t> chunk_slice; // host: n_chunks + 1 (one launch per chunk)
    int64_t *d_off = nullptr;
    int32_t *d_len = nullptr;
    int32_t *d_row = nullptr;         // row | kCcFirst, -1: no row
    uint16_t *d_row_len = nullptr;
    uint32_t *d_word = nullptr;       // column in chunk (| id << chunk_log2 in the codebook form)
    float *d_val = nullptr;           // plain form
    float *d_table = nullptr;         // codebook form
    int32_t table_size = 0;
};

// Device copy of the reference's own stream (native.hip): uint8 deltas + ids, each
// panel's run starting 16-byte aligned (padded with zero-delta fillers).
struct NatBatch {   // one batch of the native two-kernel form (16 bytes, one load)
    int64_t start;     // first entry in the padded stream
    int32_t len;       // entries (<= kNatBatchEntries)
    int32_t carry;     // in-panel offset before the batch (kernel.cc:780-781)
};

struct NativeDev {
    int32_t n_panels = 0;             // panels with entries; 0 when not built
    int32_t n_all = 0;                // + the empty 256-column blocks (beta != 1 launches)
    int64_t s_rows = 0, s_cols = 0;
    uint8_t *d_pos = nullptr, *d_val = nullptr;
    int64_t *d_beg = nullptr, *d_end = nullptr;
    int32_t *d_col = nullptr;
    float *d_table = nullptr;         // table_size raw values
    int32_t table_size = 0;
    // Two-kernel form (panels of more than kNatFusedBatches batches of 4096 entries):
    // per batch its panel and the in-panel offset before it (the reference's running
    // pos_offset, kernel.cc:780-781), per (batch, group of 64 columns) the start of its
    // column lists in d_lists (4 bytes per live entry) and per (batch, group, column)
    // the list's [begin, end) written by the decode kernel.
    int32_t n_batches = 0, max_panel_batches = 0;
    int32_t *d_pbatch = nullptr;      // n_all + 1: first batch of each panel
    NatBatch *d_bmeta = nullptr;      // per batch: stream start, entries, carry
    int32_t *d_boff = nullptr;        // per (batch, group)
    uint32_t *d_lists = nullptr;      // live entries: m = 1 the term's bits, else row | id << 23
    uint32_t *d_hdr = nullptr;        // per (batch, group, column): begin | end << 16
};
constexpr int kNatBatchEntries = 4096;
constexpr int kNatFusedBatches = 2;   // panels of at most this many batches: one fused kernel

struct SweepDev {   // column-swept row blocks (sweep.h)
    int64_t n_blocks = 0, n_chunks = 0;   // n_blocks == 0 when not built
    int64_t *d_block_chunk = nullptr;
    uint32_t *d_ent = nullptr;           // n_chunks * 128
    float *d_table = nullptr;            // 256 raw values (0 past table_size)
    int32_t table_size = 0;
};

// Merge-path SpMV, per workgroup: its first row's end part when that row began in an earlier
// workgroup (first_row >= 0), and its last row's open part (last_row >= 0; last_fresh: the
// part starts with the row's beta * y).
struct MergeRec {
    int32_t first_row;
    float first_val;
    int32_t last_row;
    float last_val;
    int32_t last_fresh;
    int32_t pad[3];
};
// The merge path's staging stream: every slice's terms in ascending column order, as
// (column << 8 | codebook id) words and their place in the slice -- so a wave's x gathers
// hit few cache lines where columns repeat (the hot, relabeled prefix of a skewed graph).
struct MergeStage {
    const uint32_t *w = nullptr;   // nnz words, slice by slice at the CSR positions [z0, z1)
    const uint16_t *z = nullptr;   // nnz positions in the slice (term z0 + z[k] of the CSR)
    const float *table = nullptr;  // 256 codebook values (0 past the table)
};
hipError_t launch_spmv_merge(int32_t n, int32_t nnz, const int32_t *rp, const int32_t *col, const float *val,
                             const float *x, float *y, float alpha, float beta, const int2 *corner, MergeRec *rec,
                             hipStream_t s, const MergeStage *stage = nullptr);

struct Plan {
    XbandDev xb;                      // n_blocks == 0 when not built
    SellDev sell;                     // n_slices == 0 when not built
    // Unsegmented sorted sliced ELL (every row, any length, in the reference's order):
    // SM_ALGO_EXACT's kernel when no other built layout keeps that order.
    SellDev xsell;
    CcsellDev cc;                     // n_slices == 0 when not built
    NativeDev nat;                    // n_panels == 0 when not built (dense-index matrices)
    SweepDev sw;                      // n_blocks == 0 when not built
    // Skewed graphs: the hottest relabeled columns [0, hot_cols) as codebook bands (x in
    // LDS), the sell layout holding only the other terms.
    XbandDev hot;                     // n_blocks == 0 when not built
    int32_t hot_cols = 0;
    int32_t tile_nnz = kTileNnz;      // one of 1024, 2048, 4096, 8192
    int32_t n_tiles = 0;
    Tile *d_tiles = nullptr;
    int32_t n_long = 0;
    int32_t *d_long_rows = nullptr;   // n_long
    int32_t *d_long_ptr = nullptr;    // n_long + 1 offsets into chunks
    int32_t n_chunks = 0;
    Chunk *d_chunks = nullptr;
    float *d_partials = nullptr;      // n_chunks long-row partial sums (one SpMV in flight)
    int32_t max_row_nnz = 0;
    double avg_row_nnz = 0.0;
    // Column relabeling for the stream kernel (skewed column degrees):
    // columns renumbered by descending number of terms, so the hot part of x is
    // a dense prefix that stays in L2.  Terms keep their stored order (bit-identical).
    int64_t n_relabel = 0;            // n_cols when built, else 0
    int32_t *d_perm = nullptr;        // original column -> new column (x is scattered)
    int32_t *d_rcol = nullptr;        // relabeled col_idx (nnz + kPadElems, zero tail)
    float *d_xperm = nullptr;         // x in the new numbering (one SpMV in flight)
    // Merge-path SpMV (kernels_merge.hip): one record per workgroup (one SpMV in flight).
    MergeRec *d_merge = nullptr;
    int2 *d_merge_corner = nullptr;   // merge_blocks + 1 slice corners
    uint32_t *d_mstage_w = nullptr;   // the merge path's column-sorted staging stream (MergeStage)
    uint16_t *d_mstage_z = nullptr;
    float *d_mstage_tab = nullptr;
};

// Host launchers (kernels.hip).  All return hipError_t of the launch.
hipError_t launch_spmv_parity(int32_t n, const int32_t *rp, const int32_t *col, const float *val,
                              const float *x, float *y, float alpha, float beta, hipStream_t s);
hipError_t launch_spmv_stream(const Plan &p, const int32_t *rp, const int32_t *col,
                              const float *val, const float *x, float *y, float alpha,
                              float beta, float *partials, hipStream_t s);
hipError_t launch_spmv_xband(const XbandDev &xb, int32_t n_rows, int32_t n_cols, const float *x,
                             float *y, float alpha, float beta, hipStream_t s);
// Sorted sliced-ELL (kernels_sell.hip): rows up to the plan's tile size.
hipError_t launch_spmv_sell(const SellDev &sd, const float *x, float *y, float alpha, float beta,
                            hipStream_t s);
// y[long_rows[i]] = beta * y + partials[long_ptr[i] .. long_ptr[i+1]) in order.
hipError_t launch_long_finalize(int32_t n_long, const int32_t *long_rows, const int32_t *long_ptr,
                                const float *partials, float *y, float beta, hipStream_t s);
// Column-chunked sorted sliced-ELL (kernels_ccsell.hip): one launch per column chunk.
hipError_t launch_spmv_sweep(const SweepDev &sd, int32_t n_rows, int32_t n_cols, const float *x,
                             float *y, float alpha, float beta, hipStream_t s);
hipError_t launch_spmv_ccsell(const CcsellDev &cd, const float *x, float *y, float alpha,
                              float beta, hipStream_t s);
// AddMatMat on the reference's stream (native.hip): C = alpha * A * S + beta * C.
hipError_t launch_native_addmatmat(const NativeDev &nd, int32_t m, const float *a, int32_t lda,
                                   float *c, int32_t ldc, float alpha, float beta, hipStream_t s);
// Balanced-band kind (kernels_band2.hip).
// Gathered chunk bands (gcb.h, kernels_gcb.hip): d_chunk_start = tile -> first band,
// d_band_clo, d_word = the lane-interleaved entries (kGcbBandWords per band).
hipError_t launch_spmv_gcb(const XbandDev &xb, int32_t n_rows, int32_t n_cols, const float *x, float *y,
                           float alpha, float beta, hipStream_t s);
hipError_t launch_spmv_band2(const XbandDev &xb, int32_t n_rows, int32_t n_cols, const float *x,
                             float *y, float alpha, float beta, hipStream_t s);
// xp[rank[c]] = x[c], c < n (rank: original column -> new column).
hipError_t launch_x_relabel(int64_t n, const int32_t *rank, const float *x, float *xp,
                            hipStream_t s);
hipError_t launch_spmv_vector(int32_t n, double avg_row, const int32_t *rp, const int32_t *col,
                              const float *val, const float *x, float *y, float alpha, float beta,
                              hipStream_t s);
// Y(j, i) = beta*Y + alpha * sum_e B[j][e] * X(col_e, i), strides given per index.
hipError_t launch_spmm_generic(int32_t n, int32_t nrhs, const int32_t *rp, const int32_t *col,
                               const float *val, const float *X, int64_t x_sk, int64_t x_si,
                               float *Y, int64_t y_sj, int64_t y_si, float alpha, float beta,
                               bool rhs_fastest, hipStream_t s);
// Row-major X (k x nrhs, ldx) / Y (n x nrhs, ldy), nrhs % 4 == 0, 16-byte aligned.
hipError_t launch_spmm_mfma(int32_t n, const int32_t *rp, const int32_t *col, const float *val,
                            int32_t nnz, const float *X, int64_t ldx, int64_t x_rows, float *Y,
                            int64_t ldy, float alpha, float beta, hipStream_t s);
hipError_t launch_spmm_rowpanel(int32_t n, int32_t nrhs, const int32_t *rp, const int32_t *col,
                                const float *val, int32_t nnz, const float *X, int64_t ldx,
                                int64_t x_rows, float *Y, int64_t ldy, float alpha, float beta,
                                bool allow_pipelined, hipStream_t s);
hipError_t launch_beta(float *c, int32_t m, int32_t n, int64_t ldc, float beta, hipStream_t s);
hipError_t launch_transpose(const float *a, int32_t m, int32_t n, int64_t lda, float *sa,
                            int64_t ldsa, hipStream_t s);
// Device CopyForm scan (encode_dev.hip).  trans: one count per index row (B row);
// otherwise one count per (chunk of chunk_rows index rows, index column), chunk-major.
hipError_t launch_encode_count(const uint8_t *dm, int32_t rows, int32_t cols, int32_t stride,
                               bool trans, int32_t chunk_rows, int32_t n_chunks, uint8_t T,
                               int32_t *cnt, hipStream_t s);
hipError_t launch_encode_fill(const uint8_t *dm, int32_t rows, int32_t cols, int32_t stride,
                              bool trans, int32_t chunk_rows, int32_t n_chunks, uint8_t T,
                              const int32_t *offs, const float *table, int32_t *col, float *val,
                              uint8_t *ids, hipStream_t s);
// The reference encoding from a device CSR (refenc_dev.hip): encode_csr_ref's result and
// return codes (encode.h), -5 on a HIP error (err).  d_ids: the terms' ids (then `table`
// is the codebook they index), else ids from the values (table, or the derived codebook).
struct EncodeResult;
int encode_csr_ref_device(const int32_t *d_rp, const int32_t *d_col, const float *d_val, const uint8_t *d_ids,
                          int64_t n_rows, int64_t n_cols, int64_t nnz, const float *table,
                          int32_t table_size, EncodeResult &out, hipStream_t s, hipError_t &err);
// Device builders (builddev.hip) on a matrix whose CSR is on the device: the column
// relabeling (check_skew: only if the top 1/16 of the columns hold >= 40 % of the terms) and
// the sorted sliced ELL (codebook form when the values allow), the bytes upload_relabel and
// upload_sell build on the host.  0 built or declined as the host would, -5 HIP error (err).
int devbuild_relabel(sm_matrix *m, bool check_skew, hipStream_t s, hipError_t &err);
int devbuild_sell(sm_matrix *m, int32_t max_len, bool codebook, hipStream_t s, hipError_t &err);
// The merge path's staging stream (merge_stage_build's bytes) from the device CSR and the
// plan's slice corners: 0 built, 1 declined as the host would, < 0 on a HIP error (err).
int devbuild_merge_stage(sm_matrix *m, hipStream_t s, hipError_t &err);
// The gathered chunk bands (builddev_gcb.hip): gcb_build's bytes into m->plan.xb's d_chunk_start,
// d_band_clo and d_word, the geometry in `meta` (its vectors stay empty).  0 built, 1 declined as
// gcb_build would, < 0 on a HIP error (err) or a builder inconsistency.
struct GcbHost;
int devbuild_gcb(sm_matrix *m, int rows_log2, int32_t n_slabs, int32_t window, GcbHost &meta, hipStream_t s,
                 hipError_t &err);
hipError_t launch_validate(int32_t n_rows, int32_t n_cols, int32_t nnz, const int32_t *rp,
                           const int32_t *col, int32_t *d_flag, hipStream_t s);
// Dense decode: out is zeroed by the caller.  b_layout: out[row*stride+col]
// (B = S^T, CopyTo Trans); else out[col*stride+row] (S, CopyTo NoTrans).
hipError_t launch_scatter_dense(int32_t n, const int32_t *rp, const int32_t *col,
                                const float *val, float *out, int64_t stride, bool b_layout,
                                hipStream_t s);
hipError_t launch_panel_kernel(int variant, int32_t m, int32_t n, int32_t k, const float *a,
                               int32_t lda, float *c, int32_t ldc, float alpha,
                               const uint8_t *ppos, const uint8_t *pval, int32_t pos_len,
                               const float *table, int32_t valid_table_size, void *workspace,
                               hipStream_t s);
size_t panel_kernel_workspace_bytes(int32_t pos_len, int32_t n);

}  // namespace smamd

// The opaque handle.
struct sm_matrix {
    int32_t device = 0;
    int64_t n_rows = 0, n_cols = 0, nnz = 0;   // CSR of B = S^T
    int64_t s_rows = 0, s_cols = 0;            // reference S view
    int32_t *d_row_ptr = nullptr;
    int32_t *d_col = nullptr;
    float *d_val = nullptr;
    smamd::Plan plan;
    smamd::BuildOpts opts;                     // layout options the matrix was built with
    int64_t device_bytes = 0;
    // Reference encoding (only for matrices built by sm_create_from_dense_index).
    bool has_ref = false;
    bool from_index = false;   // built by the CopyForm constructors (the reference's path)
    int32_t table_size = 0;
    std::vector<float> table;                  // table_size + 1, last = 0
    std::vector<uint8_t> pos, val;
    std::vector<int32_t> panel_row_off, panel_col_off;
    std::vector<int64_t> panel_begin, panel_end;
    // Workspace of the row-panel AddMatMat (sm_addmatmat, 2 <= m <= 128), kept across
    // calls.  Each call makes its stream wait on ws_ready (recorded after the previous
    // call's last kernel), so calls on any streams use it in turn; it grows (after its
    // last user has drained) only when a call needs more.
    mutable std::mutex ws_mu;
    mutable float *d_ws = nullptr;
    mutable size_t ws_bytes = 0;
    mutable hipEvent_t ws_ready = nullptr;
    // SpMV scratch (slab partials and hand-off words, long-row partials, the relabeled
    // x) belongs to the matrix: every SpMV that uses it makes its stream wait on
    // scratch_ready (recorded after the previous such SpMV's kernels), so SpMVs on one
    // matrix from several streams or threads run one after the other on the device,
    // correct, the way the reference's read-only AddMatMat allows concurrent callers
    // (sparse-matrix.cc:139-194).  Calls into a stream being captured are ordered by
    // that stream alone.
    mutable std::mutex scratch_mu;
    mutable hipEvent_t scratch_ready = nullptr;
    mutable bool scratch_recorded = false;
};
