/*
 * sparsematrix.h -- C ABI of sparsematrix_amd (libsparsematrix_amd.so), an
 * MI355X-native (gfx950) replacement for NeverLEX/sparsematrix's sparse x dense
 * multiply.  Plain pointers and sizes only; no C++ or torch types.
 *
 * Orientation.  The reference stores S (k x n) and computes, for a dense
 * row-major A (m x k) and C (m x n),  C = alpha*A*S + beta*C
 * (sparse-matrix.h:37, sparse-matrix.cc:139-194).  Here the matrix is held on
 * the device as CSR of B = S^T (n rows x k columns, int32 row_ptr/col_idx,
 * fp32 values), so m = 1 is the SpMV  y = alpha*B*x + beta*y  and a panel of
 * N right-hand sides is the SpMM  Y = alpha*B*X + beta*Y  (X: k x N, Y: n x N,
 * both row-major).  sm_num_rows/sm_num_cols report the reference's S view
 * (rows_ = k, cols_ = n; sparse-matrix.h:39-40).
 *
 * Semantics kept from the reference (SURVEY.md §7 "Drop-in semantics"):
 *   - beta is applied by multiplication whenever beta != 1 (so beta = 0
 *     propagates NaN/Inf already in C/y)                 kernel.cc:10-29
 *   - alpha == 0 skips the product entirely              sparse-matrix.cc:152
 *   - alpha is folded into the stored value first: each term is
 *     x * (v * alpha), added one at a time               kernel.cc:791, 580-582
 *   - ids >= table_size are not stored; explicit 0.0 table entries are
 *                                                        sparse-matrix.cc:44, 77
 * Summation order: SM_ALGO_PARITY adds the terms of every output in stored
 * (ascending column) order, exactly as the reference does, so results are
 * bit-identical to the reference CPU kernel.  SM_ALGO_XBAND keeps that order for
 * every row on the exact band layout (sm_info.has_xband == 1, or any layout with
 * xband_slabs == 1); the slab layouts (has_xband 2-5) sum each column slab in
 * order and add the slab sums in slab order (band2 / cband after beta*y:
 * sm_info.xband_beta_last).  SM_ALGO_SELL keeps it for every row
 * of up to 2048 terms and adds longer rows' 2048-term segment sums in order.  The
 * SpMM kernels keep it for every row.  SM_ALGO_STREAM keeps it for rows of up to
 * SM_SERIAL_ROW_MAX terms and uses a tree sum for longer rows.  The bound for
 * every non-exact case is |y - y_ref| <= 1e-6 * sum|terms|.
 *
 * Concurrency: calls on one matrix from several streams or threads are correct;
 * SpMVs that use the matrix's scratch take turns on the device.
 *
 * Errors: every call returns sm_status; sm_last_error() gives a message for
 * the calling thread.  Device calls are asynchronous on `stream` (a
 * hipStream_t; NULL = the legacy default stream) unless stated otherwise.
 */
#ifndef SPARSEMATRIX_AMD_H
#define SPARSEMATRIX_AMD_H

#include <stddef.h>
#include <stdint.h>

#if defined(__GNUC__)
#define SM_API __attribute__((visibility("default")))
#else
#define SM_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

typedef enum sm_status {
    SM_OK = 0,
    SM_ERR_INVALID_ARG = 1,     /* bad shape, stride, pointer or enum          */
    SM_ERR_OUT_OF_MEMORY = 2,   /* host or device allocation failed            */
    SM_ERR_HIP = 3,             /* a HIP runtime call failed                   */
    SM_ERR_NOT_SUPPORTED = 4,   /* operation not available for this matrix     */
    SM_ERR_TOO_LARGE = 5,       /* exceeds int32 indexing (nnz or rows >= 2^31) */
    SM_ERR_INVALID_MATRIX = 6,  /* CSR failed validation (col out of range...) */
    SM_ERR_NO_DEVICE = 7        /* no HIP device visible                       */
} sm_status;

/* SBLAS_TRANSPOSE, sparse-matrix.h:20-23 */
typedef enum sm_trans { SM_NO_TRANS = 0, SM_TRANS = 1 } sm_trans;

typedef enum sm_algo {
    SM_ALGO_AUTO = 0,     /* band layout if built, else sell, else stream (SpMV); row-panel (SpMM) */
    SM_ALGO_PARITY = 1,   /* bit-exact with the reference for every row            */
    SM_ALGO_STREAM = 2,   /* nnz-balanced row tiles through LDS (+ long-row split) */
    SM_ALGO_VECTOR = 3,   /* L lanes per row (CSR-vector), shuffle reduction       */
    SM_ALGO_XBAND = 4,    /* x staged through LDS in column bands (the layout built at
                             creation, see sm_info.has_xband); falls back to SELL, then
                             STREAM, when the matrix holds no band layout             */
    SM_ALGO_SELL = 5,     /* sorted sliced-ELL, one lane per row (every row up to 2048
                             terms bit-identical; longer rows in 2048-term segments whose
                             sums are added in order); STREAM when not built           */
    SM_ALGO_NATIVE = 6,   /* the reference's own stream (uint8 deltas + ids, 256-column
                             panels) decoded on the device; bit-identical for every
                             output; only for matrices built from the dense index
                             (SM_ERR_NOT_SUPPORTED otherwise)                          */
    SM_ALGO_EXACT = 7,    /* the fastest kernel built for the matrix that adds every
                             output's terms in the reference's order (bit-identical):
                             the column-swept or one-slab band layout, the column-chunked
                             or segment-free sliced ELL, the stream kernel when no row
                             exceeds SM_SERIAL_ROW_MAX terms, else PARITY.  SpMM and
                             AddMatMat with m > 1: the row-panel kernels (every row in
                             order).  What the reference's C++ surface (libsblas) runs. */
    SM_ALGO_MFMA = 8,     /* SpMM with n_rhs == 32 only: 16-row tiles on the matrix cores
                             (v_mfma_f32_16x16x4_f32, four terms per step), one fused
                             multiply-add per term: within the sum|terms| bound, not
                             bit-identical; X must be finite (a non-finite X row makes
                             the tile's other outputs NaN).  SM_ERR_NOT_SUPPORTED for
                             other shapes and for SpMV.                                */
    SM_ALGO_MERGE = 9     /* SpMV by merge path (Merrill & Garland): every workgroup and
                             thread an equal share of rows + terms, rows cut anywhere.
                             A row inside one thread's share is summed in stored order
                             (bit-identical); cut rows join their parts in a fixed order
                             (within the sum|terms| bound, deterministic).  SpMM: as AUTO. */
} sm_algo;

/* Rows with at most this many terms are summed in reference order by the
 * fast kernels (bit-exact); longer rows use a tree reduction. */
#define SM_SERIAL_ROW_MAX 64

typedef struct sm_matrix sm_matrix;   /* opaque, device-resident */
typedef void *sm_stream;              /* hipStream_t */

typedef struct sm_info {
    int64_t s_rows, s_cols;     /* reference S view: rows_ = k, cols_ = n      */
    int64_t n_rows, n_cols;     /* CSR of B = S^T: n rows, k columns          */
    int64_t nnz;                /* stored entries (explicit zeros included)    */
    int32_t table_size;         /* codebook size T (0 if built from CSR)       */
    int32_t has_ref_stream;     /* 1 if the reference encoding is held         */
    int64_t n_entries;          /* reference stream length (nnz + fillers)     */
    int64_t n_panels;           /* reference panels (block_bounds_.size())     */
    int32_t device;             /* HIP device ordinal holding the matrix       */
    int32_t n_tiles;            /* stream-kernel row tiles                     */
    int32_t n_long_rows;        /* rows split across workgroups                */
    int32_t max_row_nnz;        /* longest row                                 */
    int32_t has_xband;          /* column-band layout: 0 none, 1 exact (bit-identical),
                                   2 blocked, 3 gather, 4 band2 (balanced bands),
                                   5 cband (balanced bands, codebook words),
                                   6 gcb (gathered chunk bands);
                                   2-6 sum each column slab in the reference's
                                   order and add the slab sums in slab order     */
    int32_t xband_blocks, xband_bands;
    int32_t xband_slabs;        /* column slabs per row block (1: bit-identical) */
    int32_t xband_block_rows;   /* rows per block                              */
    int64_t device_bytes;       /* device memory held by the matrix            */
    int32_t col_relabel;        /* 1: the stream SpMV gathers x through a column
                                   relabeling by descending degree (skewed graphs) */
    int32_t xband_slab_cols;    /* columns per slab (slab s = [s*c, (s+1)*c))   */
    int64_t sell_slices;        /* sorted sliced-ELL slices of 64 rows (0: not built) */
    int32_t sell_codebook;      /* 1: the slices hold 4-byte column | codebook-id words */
    int32_t ccsell_chunks;      /* column chunks of the column-chunked sliced ELL (0: not built);
                                   it serves SpMV when built (AUTO, SELL): every row bit-identical */
    int32_t hot_cols;           /* > 0: the relabeled columns [0, hot_cols) run as codebook bands
                                   before the sliced ELL adds the other terms (AUTO, SELL)  */
    int32_t sweep_blocks;       /* row blocks of the column-swept layout (0: not built); it
                                   serves SpMV when built (AUTO): every row bit-identical    */
    int64_t exact_sell_slices;  /* slices of the unsegmented sliced ELL (sm_build_opts.exact_sell;
                                   0: not built) that SM_ALGO_EXACT runs                   */
    int32_t exact_algo;         /* the sm_algo SM_ALGO_EXACT runs for a 16-byte aligned x
                                   (SM_ALGO_SELL also for the unsegmented sliced ELL)       */
    int32_t xband_slab0_cols;   /* columns of slab 0 (slab s >= 1 covers [slab0 + (s-1) *
                                   xband_slab_cols, slab0 + s * xband_slab_cols)); equal to
                                   xband_slab_cols when the slabs are even                  */
    int32_t merge_stage;        /* 1: SM_ALGO_MERGE stages terms from the column-sorted copy
                                   (sm_build_opts.merge_stage)                               */
    int32_t xband_beta_last;    /* 1: the slab sums are added after beta*y -- y = (((beta*y +
                                   P_0) + P_1) + ...), every P_s summed from -0.0 (band2 / cband
                                   with several slabs); 0: slab 0 starts from beta*y          */
} sm_info;

/* ---- library ----------------------------------------------------------- */
SM_API const char *sm_version(void);
SM_API const char *sm_status_string(sm_status s);
SM_API const char *sm_last_error(void);
SM_API sm_status sm_device_count(int32_t *count);

/* ---- construction ---------------------------------------------------------
 * sm_create_from_dense_index: replaces SparseMatrix::CopyForm
 * (sparse-matrix.cc:20-99; ctor sparse-matrix.h:29-31).  `index` is a
 * rows x stride uint8 matrix of codebook ids; ids >= table_size are empty.
 * NoTrans: S = index (rows x cols).  Trans: S = index^T (cols x rows).
 * table_size must be in [0, 255]; 0 yields an empty 0 x 0 matrix
 * (sparse-matrix.cc:25-26).  Host pointers; the CSR is uploaded to `device`. */
SM_API sm_status sm_create_from_dense_index(const uint8_t *index, int32_t rows, int32_t cols,
                                            int32_t stride, const float *table,
                                            int32_t table_size, sm_trans trans,
                                            int32_t device, sm_matrix **out);

/* Same as sm_create_from_dense_index with the index already on `device`
 * (`d_index`, rows x stride bytes; `table` stays a host pointer): the scan runs
 * on the device (count, host prefix sum, fill) and yields
 * the same CSR bit for bit.  No reference stream is kept, so sm_copy_ref_stream
 * does not apply.  Synchronises `stream`. */
SM_API sm_status sm_create_from_dense_index_device(const uint8_t *d_index, int32_t rows,
                                                   int32_t cols, int32_t stride,
                                                   const float *table, int32_t table_size,
                                                   sm_trans trans, int32_t device,
                                                   sm_stream stream, sm_matrix **out);

/* Additive CSR ingestion (no reference equivalent: the reference cannot encode
 * the north-star sizes).  B is n_rows x n_cols; row_ptr has
 * n_rows+1 entries.  Host pointers, validated on the host. */
SM_API sm_status sm_create_from_csr(int64_t n_rows, int64_t n_cols, int64_t nnz,
                                    const int32_t *row_ptr, const int32_t *col_idx,
                                    const float *val, int32_t device, sm_matrix **out);

/* Same, from device pointers on `device` (copied device-to-device on `stream`
 * and validated by a kernel; synchronises `stream`).  The layout builders run on
 * the host: the columns (and, for the layout that stores them, the values) are
 * copied to the host once, at creation -- 4 + 4 bytes per term over PCIe. */
SM_API sm_status sm_create_from_csr_device(int64_t n_rows, int64_t n_cols, int64_t nnz,
                                           const int32_t *d_row_ptr, const int32_t *d_col_idx,
                                           const float *d_val, int32_t device, sm_stream stream,
                                           sm_matrix **out);

/* ---- layout options ---------------------------------------------------------
 * The constructors pick the SpMV layout themselves (SM_LAYOUT_AUTO).
 * sm_create_from_csr_ex / _device_ex take these options instead, to force a layout
 * (tests, A/B measurements).  Every layout computes the same product; they differ
 * in speed and in where the bit-exact reference order holds (sm_info.has_xband).
 * Fields past `struct_size` keep their defaults, so callers built against an
 * older header stay valid.  Initialise with sm_build_opts_init. */
typedef enum sm_layout {
    SM_LAYOUT_AUTO = 0,      /* cost model: balanced codebook bands / bands / sell / stream */
    SM_LAYOUT_EXACT = 1,     /* column bands, one slab: every row in the reference's order */
    SM_LAYOUT_BLOCKED = 2,   /* column bands in slabs (x staged through LDS)               */
    SM_LAYOUT_GATHER = 3,    /* column-ordered bands, x gathered                           */
    SM_LAYOUT_BAND2 = 4,     /* balanced bands, 8-byte entries                             */
    SM_LAYOUT_CBAND = 5,     /* balanced bands, 4-byte codebook words                      */
    SM_LAYOUT_NO_BANDS = 6,  /* no band layout: sorted sliced-ELL, else the stream kernel   */
    SM_LAYOUT_BANDS = 7,     /* a band layout even where the cost model would decline; the
                                kind as AUTO would pick it                                */
    SM_LAYOUT_SWEEP = 8,     /* column-swept row blocks (wide matrices, <= 255 values): one
                                wavefront per 256 rows, terms in column order, no barrier  */
    SM_LAYOUT_GCB = 9        /* gathered chunk bands (wide matrices, x far beyond L2): 32K-row
                                tiles, bands of up to 2016 terms within 2^18 columns, x
                                gathered per term, rows' sums in LDS                      */
} sm_layout;

typedef struct sm_build_opts {
    int32_t struct_size;       /* sizeof(sm_build_opts) as the caller compiled it      */
    int32_t layout;            /* sm_layout                                            */
    int32_t band_slabs;        /* balanced bands: column slabs per row block, 0 = auto  */
    int32_t band_tall;         /* balanced-band geometry: 0 or 4 = dma3 (a loader wave
                                  stages x by LDS-DMA into three 7680-column buffers; the
                                  default), 6 = wide (8192-column windows staged by every
                                  wave); other values are SM_ERR_INVALID_ARG            */
    int32_t gather_band_log2;  /* gather bands: 13, 14 or 15 (log2 columns), 0 = auto  */
    int32_t sell;              /* sorted sliced-ELL: -1 auto (built when no band layout), 0 never */
    int32_t sell_codebook;     /* sell slots as column|id words: -1 auto, 0 never      */
    int32_t sell_max_len;      /* rows longer than this are cut in segments, 0 = 2048  */
    int32_t sell_streams;      /* XCD streams of sort windows, 0 = auto                */
    int64_t sell_sigma;        /* sort rows by length within windows of this many rows, 0 = globally */
    int32_t relabel;           /* column relabeling by degree: -1 auto, 0 never, 1 always */
    int32_t tile_nnz;          /* stream-kernel tile: 1024/2048/4096/8192, 0 = auto   */
    int32_t ccsell;            /* column-chunked sliced-ELL (wide x): -1 auto, 0 never, 1 always
                                  (where no band layout is built and it applies)       */
    int32_t ccsell_chunk_log2; /* its column chunk, log2 columns (8..24), 0 = 20 (4 MiB of x) */
    int32_t hot_cols;          /* skewed graphs (column relabeling built), opt-in: > 0 sends the
                                  hottest this many relabeled columns through codebook bands
                                  with x in LDS, the rest through the sliced ELL (within the
                                  Sum|terms| bound); 0 / -1 never (slower on R-MAT 24)     */
    int32_t exact_sell;        /* an unsegmented sorted sliced ELL beside the layout above, for
                                  SM_ALGO_EXACT when no built layout keeps the reference's order
                                  for every row: 0 auto (matrices from the dense index, i.e.
                                  the reference's CopyForm path), 1 always, -1 never        */
    int32_t band_slab0_permille; /* balanced bands with several slabs: slab 0's columns as a
                                  share of an even split, in permille (0 = auto = 1000, even
                                  slabs); the other slabs share the rest evenly.  The slab-0
                                  tile also loads and scales y before its first band        */
    int32_t merge_stage;       /* SM_ALGO_MERGE on skewed graphs: 1 builds a column-sorted copy of
                                  each merge tile's terms (4-byte column | codebook-id words and
                                  2-byte slots, 6 bytes per term) when the values form a codebook
                                  and n_cols <= 2^24; the tile gathers x in column order (R-MAT 24:
                                  1.91 -> 1.68 ms), same bits as without.  0 = never (default)  */
    int32_t host_build;        /* sm_create_from_csr_device: 0 = auto -- the column relabeling and
                                  the sorted sliced ELL are built on the device where they are
                                  the only layouts wanted (builddev.hip; the same bytes as the
                                  host builders); 1 = always on the host                      */
} sm_build_opts;

SM_API void sm_build_opts_init(sm_build_opts *opts);

SM_API sm_status sm_create_from_csr_ex(int64_t n_rows, int64_t n_cols, int64_t nnz,
                                       const int32_t *row_ptr, const int32_t *col_idx,
                                       const float *val, int32_t device,
                                       const sm_build_opts *opts, sm_matrix **out);
SM_API sm_status sm_create_from_csr_device_ex(int64_t n_rows, int64_t n_cols, int64_t nnz,
                                              const int32_t *d_row_ptr, const int32_t *d_col_idx,
                                              const float *d_val, int32_t device,
                                              sm_stream stream, const sm_build_opts *opts,
                                              sm_matrix **out);

/* Destroy: sparse-matrix.cc:9-18 (frees host and device storage). */
SM_API void sm_destroy(sm_matrix *m);

/* ---- queries ----------------------------------------------------------- */
/* sm_info grew in 0.2 (xband_slab_cols, sell_slices, sell_codebook): a caller built
 * against an older header passes its own sizeof to sm_get_info_ex, which writes only
 * that many bytes.  sm_get_info writes the whole struct of this header. */
SM_API sm_status sm_get_info(const sm_matrix *m, sm_info *info);
SM_API sm_status sm_get_info_ex(const sm_matrix *m, sm_info *info, size_t info_bytes);
/* Diagnostics: 64-bit FNV-1a digests of the device layout arrays, so two builds can be
 * compared byte for byte (sm_build_opts.host_build): [0] the column relabeling (new column
 * of every original column, relabeled col_idx), [1] the sorted sliced ELL's structure
 * (slice offsets and lengths, lane rows and lengths, long rows and their partial offsets),
 * [2] its slots (column words, values), [3] its codebook and the merge path's staging copy
 * (sm_build_opts.merge_stage: column words, offsets, table).  0 for a part not built.  With the
 * gathered chunk bands (SM_LAYOUT_GCB) [1] is their geometry, tile -> band offsets and band
 * start columns, [2] the bands' words.  Synchronises the device. */
SM_API sm_status sm_layout_digest(const sm_matrix *m, uint64_t digest[4]);
SM_API int32_t sm_num_rows(const sm_matrix *m);   /* NumRows, sparse-matrix.h:39 */
SM_API int32_t sm_num_cols(const sm_matrix *m);   /* NumCols, sparse-matrix.h:40 */

/* The reference encoding (sparse-matrix.h:46-52): E delta steps and ids, and
 * per panel (row_off, col_off, begin, end).  Sizes from sm_get_info. */
SM_API sm_status sm_copy_ref_stream(const sm_matrix *m, uint8_t *pos, uint8_t *val,
                                    int32_t *panel_row_off, int32_t *panel_col_off,
                                    int64_t *panel_begin, int64_t *panel_end);

/* The reference encoding of a matrix built from CSR (sm_create_from_csr*, or the
 * device CopyForm scan), built on the host from its CSR by the reference's own stream
 * rules (sparse-matrix.cc:20-99: 256-column panels, row-major, uint8 delta steps with
 * (255, T) fillers, uint8 ids): afterwards sm_copy_ref_stream, sm_equal's member-wise
 * comparison and SM_ALGO_NATIVE serve the matrix.  `table` (table_size <= 255 entries)
 * is the codebook every value must match bit for bit (the first equal entry's id);
 * NULL takes the values' distinct bit patterns in CSR order (SM_ERR_NOT_SUPPORTED past
 * 255).  A matrix that already holds the encoding is left as it is.  Not concurrent with
 * other calls on the matrix.  Additive: the reference cannot hold a matrix without it. */
SM_API sm_status sm_build_ref_stream(sm_matrix *m, const float *table, int32_t table_size);

/* Host copy of the device CSR (row_ptr n_rows+1, col_idx/val nnz). */
SM_API sm_status sm_copy_csr(const sm_matrix *m, int32_t *row_ptr, int32_t *col_idx, float *val);

/* CopyTo (sparse-matrix.cc:101-137), host output.  NoTrans writes S
 * (s_rows x stride), Trans writes S^T (s_cols x stride); untouched elements
 * are zeroed.  Decoded on the device. */
SM_API sm_status sm_to_dense(const sm_matrix *m, float *out, int32_t stride, sm_trans trans);

/* operator== (sparse-matrix.cc:197-207) on semantic content: shape, stored
 * (row, col, value) triples and, for codebook matrices, the table. */
SM_API int32_t sm_equal(const sm_matrix *a, const sm_matrix *b);

/* ---- compute on device pointers ----------------------------------------- */
/* y[n_rows] = alpha * B * x[n_cols] + beta * y */
SM_API sm_status sm_spmv(const sm_matrix *m, float alpha, const float *x, float beta, float *y,
                         sm_algo algo, sm_stream stream);

/* Y (n_rows x n_rhs, ldy) = alpha * B * X (n_cols x n_rhs, ldx) + beta * Y */
SM_API sm_status sm_spmm(const sm_matrix *m, int32_t n_rhs, float alpha, const float *X,
                         int64_t ldx, float beta, float *Y, int64_t ldy, sm_algo algo,
                         sm_stream stream);

/* AddMatMat (sparse-matrix.cc:139-194) on device pointers:
 * C (m x n, ldc) = alpha * A (m x k, lda) * S + beta * C.
 * m = 1: sm_spmv.  2 <= m <= 128 with algo != SM_ALGO_PARITY: transposes + row-panel
 * SpMM in the matrix's workspace, asynchronous on `stream`: the stream first waits on
 * an event recorded after the previous call's last use of the workspace (calls from
 * any streams take turns on the device; the host blocks only when a larger m makes
 * the workspace grow); m > 128: the same per group of 128 rows of A and C.
 * SM_ALGO_PARITY: one thread per output reads A and C in place. */
SM_API sm_status sm_addmatmat(const sm_matrix *mat, const float *a, int32_t m, int32_t lda,
                              float *c, int32_t ldc, float alpha, float beta, sm_algo algo,
                              sm_stream stream);

/* Synchronous drop-in for AddMatMat on HOST pointers (uploads A and C, computes with
 * SM_ALGO_EXACT, downloads C).  Bit-identical to the reference. */
SM_API sm_status sm_addmatmat_host(const sm_matrix *mat, const float *a, int32_t m, int32_t lda,
                                   float *c, int32_t ldc, float alpha, float beta);

/* ---- kernel.h helpers (kernel.cc:10-187), device pointers ---------------- */
/* c[i*ldc + j] *= beta for i < m, j < n */
SM_API sm_status sm_beta_scale(float *c, int32_t m, int32_t n, int32_t ldc, float beta,
                               sm_stream stream);
/* sa[j*ldsa + i] = a[i*lda + j] for i < m, j < n (out of place) */
SM_API sm_status sm_transpose(const float *a, int32_t m, int32_t n, int32_t lda, float *sa,
                              int32_t ldsa, sm_stream stream);

/* ---- reference-format panel kernels (kernel.h:42-62), device pointers -----
 * One panel of the reference stream (ppos/pval, pos_len entries; positions
 * are row*256 + col inside the panel), codebook `table` of valid_table_size+1
 * floats.  variant: 0 = sblas_kernel_operation, 1 = _naive (A m x k lda,
 * C m x n ldc), 2 = _trans, 3 = _trans_ex (A^T k x lda, C^T n x ldc). */
SM_API sm_status sm_panel_kernel(int32_t variant, int32_t m, int32_t n, int32_t k,
                                 const float *a, int32_t lda, float *c, int32_t ldc, float alpha,
                                 const uint8_t *ppos, const uint8_t *pval, int32_t pos_len,
                                 const float *table, int32_t valid_table_size, sm_stream stream);

/* Synchronise the stream and report asynchronous kernel errors. */
SM_API sm_status sm_stream_sync(sm_stream stream);

/* Testing hook: set the slab hand-off launch counter of every row block of a band2 /
 * cband layout (xband_dev.h, 64-bit, monotonic) to `started` and clear its arrival
 * words, as if `started` tiles had run before -- e.g. 2^32 - 1 to run launches across
 * the 32-bit boundary.  Synchronous; no SpMV on the matrix may be in flight.
 * SM_ERR_NOT_SUPPORTED when the matrix has no multi-slab band2 / cband layout, or when
 * `started` is not a whole number of launches (a multiple of the slab count). */
SM_API sm_status sm_debug_seed_handoff(sm_matrix *m, uint64_t started);

/* ---- multi-GPU: row partition + one RCCL all-gather per product ------------
 * SURVEY.md §8(e).  One process per GPU of one node.  Rank r holds its rows of B
 * (any contiguous split; sm_multi_partition gives the equal one) as an sm_matrix with
 * GLOBAL column indices, so its n_cols is the global column count.  x is split in
 * nranks equal slices (n_cols % nranks == 0): rank r supplies x[r*L, (r+1)*L),
 * L = n_cols / nranks.  Per product the only exchange is one ncclAllGather of the x
 * slices (SpMM: of the X panel's row slices) over xGMI into the context's buffer,
 * then the local SpMV / SpMM on the same stream.  No other collective: the reference's
 * panels already write disjoint outputs (sparse-matrix.cc:164-190).
 * RCCL is loaded at run time (the copy already in the process if any, else
 * $SM_RCCL_LIB if set, else the system's); without it sm_multi_create returns
 * SM_ERR_NOT_SUPPORTED (sm_multi_create_with takes any all-gather instead).
 * Errors: sm_multi_last_error(). */
#define SM_UNIQUE_ID_BYTES 128
typedef struct sm_unique_id { char internal[SM_UNIQUE_ID_BYTES]; } sm_unique_id;
typedef struct sm_multi sm_multi;

SM_API const char *sm_multi_last_error(void);
/* Rows [r0, r1) of rank `rank` in the equal split of n rows (the first n % nranks ranks
 * get one row more).  Pure arithmetic, no device. */
SM_API sm_status sm_multi_partition(int64_t n, int32_t nranks, int32_t rank, int64_t *r0,
                                    int64_t *r1);
/* Rank 0 creates the id and passes it to every rank out of band (MPI, a file,
 * torch.distributed). */
SM_API sm_status sm_multi_unique_id(sm_unique_id *id);
/* Collective: every rank calls it with the same id and nranks.  The context refers to
 * `local` (not owned; keep it alive) and joins the communicator on its device. */
SM_API sm_status sm_multi_create(const sm_unique_id *id, int32_t nranks, int32_t rank,
                                 const sm_matrix *local, sm_multi **out);
/* A caller-supplied all-gather instead of RCCL (no reference equivalent: the reference
 * has no multi-device path).  `allgather` gathers `count` floats from every rank's
 * `send` into `recv` in rank order (rank r's slice at recv + r*count), ordered on
 * `stream` (a hipStream_t): it may enqueue device work on `stream`, or synchronise
 * `stream` and block the host until `recv` holds the result (a host-staged gather over
 * MPI, gloo, ...).  It returns 0 on success.  Everything else -- the partition, the two
 * gather buffers, their stream ordering, the pipelined batch -- is the context's, as
 * with RCCL.  sm_multi_unique_id is not needed. */
typedef int32_t (*sm_allgather_fn)(const float *send, float *recv, int64_t count,
                                   sm_stream stream, void *user);
typedef struct sm_collective {
    sm_allgather_fn allgather;
    void *user;   /* passed back to every call */
} sm_collective;
SM_API sm_status sm_multi_create_with(const sm_collective *coll, int32_t nranks, int32_t rank,
                                      const sm_matrix *local, sm_multi **out);
SM_API void sm_multi_destroy(sm_multi *mc);
/* y_local = alpha * B_local * x + beta * y_local, x = all-gather of the x_local slices. */
SM_API sm_status sm_multi_spmv(sm_multi *mc, float alpha, const float *x_local, float beta,
                               float *y_local, sm_algo algo, sm_stream stream);
/* Y_local (rows x n_rhs, ldy) = alpha * B_local * X + beta * Y_local; X_local is this
 * rank's L x n_rhs row-major slice of X (contiguous, ldx = n_rhs). */
SM_API sm_status sm_multi_spmm(sm_multi *mc, int32_t n_rhs, float alpha, const float *X_local,
                               float beta, float *Y_local, int64_t ldy, sm_algo algo,
                               sm_stream stream);
/* `count` independent products y_local[i] = alpha * B_i * x + beta * y_local[i], x the
 * all-gather of x_local[i], B_i = locals[i] (NULL: the context's matrix; others must
 * have the same global columns and device): the all-gather of product i+1 runs on the
 * context's own stream beside the SpMV of product i on `stream` (two gather buffers
 * alternate); still one all-gather per product.  Returns with the whole batch ordered
 * before later work on `stream`. */
SM_API sm_status sm_multi_spmv_batch(sm_multi *mc, int32_t count, const sm_matrix *const *locals,
                                     float alpha, const float *const *x_local, float beta,
                                     float *const *y_local, sm_algo algo, sm_stream stream);
/* The all-gather alone (n_rhs = 1 for x), into the context's buffer; *x_full (optional)
 * receives its device address, valid until the next call on the context (which waits
 * for the work queued on `stream` up to this call, not for reads the caller adds later
 * on other streams).
 * Buffer ordering: every product records, on the stream that ran it, that it has read
 * the gathered x; any later all-gather into that buffer waits for it, from whatever
 * stream.  Calls on one context therefore may come from several streams.  Inside a
 * stream capture, the captured products are ordered by the capture only: a graph replay
 * is not tracked, so the caller orders replays of captured products against eager calls
 * on other streams (an event after each replay).  A capture cannot grow the gather
 * buffers (that needs a device sync): a captured product larger than every earlier one
 * fails with SM_ERR_NOT_SUPPORTED -- run one eager product of that size first. */
SM_API sm_status sm_multi_allgather(sm_multi *mc, const float *x_local, int32_t n_rhs,
                                    sm_stream stream, const float **x_full);
/* Device timing of sm_multi_spmv / _spmm (HIP events around the all-gather and the
 * local product); sm_multi_last_times waits for the last call and reports both. */
SM_API sm_status sm_multi_set_timing(sm_multi *mc, int32_t on);
SM_API sm_status sm_multi_last_times(sm_multi *mc, float *allgather_ms, float *compute_ms);

#ifdef __cplusplus
}
#endif
#endif /* SPARSEMATRIX_AMD_H */
