/*
 * oracle/refmodel.c -- TEST INFRASTRUCTURE ONLY (see refmodel.h).
 *
 * Clean-room C restatement of the reference's hot path.  Every function cites
 * the reference lines (paths relative to /root/reference) whose behaviour it
 * restates.  Compiled with -O2 -ffp-contract=off (oracle/Makefile).
 */
#include "refmodel.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define PANEL_SHIFT 8                      /* SBLAS_BLOCK_COL_SHIFT, kernel.h:26 */
#define PANEL_W     (1 << PANEL_SHIFT)     /* 256 columns per panel */
#define PANEL_MASK  (PANEL_W - 1)
#define MAX_STEP    255                    /* uint8 delta range, sparse-matrix.cc:24 */

/* ---- growable byte streams -------------------------------------------- */
typedef struct { uint8_t *pos, *val; int64_t n, cap; } stream_t;

static int stream_push(stream_t *s, uint8_t p, uint8_t v) {
    if (s->n == s->cap) {
        int64_t cap = s->cap ? s->cap * 2 : 1024;
        uint8_t *np = (uint8_t *)realloc(s->pos, (size_t)cap);
        if (!np) return -1;
        s->pos = np;
        uint8_t *nv = (uint8_t *)realloc(s->val, (size_t)cap);
        if (!nv) return -1;
        s->val = nv;
        s->cap = cap;
    }
    s->pos[s->n] = p;
    s->val[s->n] = v;
    s->n++;
    return 0;
}

typedef struct { int32_t *ro, *co; int64_t *b, *e; int32_t n, cap; } panels_t;

static int panels_push(panels_t *p, int32_t ro, int32_t co, int64_t b, int64_t e) {
    if (p->n == p->cap) {
        int32_t cap = p->cap ? p->cap * 2 : 16;
        p->ro = (int32_t *)realloc(p->ro, sizeof(int32_t) * cap);
        p->co = (int32_t *)realloc(p->co, sizeof(int32_t) * cap);
        p->b = (int64_t *)realloc(p->b, sizeof(int64_t) * cap);
        p->e = (int64_t *)realloc(p->e, sizeof(int64_t) * cap);
        if (!p->ro || !p->co || !p->b || !p->e) return -1;
        p->cap = cap;
    }
    p->ro[p->n] = ro; p->co[p->n] = co; p->b[p->n] = b; p->e[p->n] = e;
    p->n++;
    return 0;
}

/* One stored entry at in-panel linear position `lin` (= srow*256 + pcol):
 * emit 255-steps with the filler id until the remaining gap fits a byte
 * (sparse-matrix.cc:44-52 / 77-85). */
static int emit_entry(stream_t *s, int32_t *prev, int32_t lin, uint8_t id, uint8_t filler) {
    int32_t gap = lin - *prev;
    while (gap > MAX_STEP) {
        if (stream_push(s, MAX_STEP, filler)) return -1;
        gap -= MAX_STEP;
    }
    if (stream_push(s, (uint8_t)gap, id)) return -1;
    *prev = lin;
    return 0;
}

/* CopyForm, sparse-matrix.cc:20-99.  With block_row_shift == 0 there is a
 * single row block spanning every S-row, and panels of 256 S-columns.
 *   NoTrans: S = dm (rows x cols), S[r][c] = dm[r*stride + c]      (:32-62)
 *   Trans:   S = dm^T (cols x rows), S[r][c] = dm[c*stride + r]    (:65-97)
 * Entries whose id >= table_size are not stored (:44, :77). */
int om_encode(const uint8_t *dm, int32_t rows, int32_t cols, int32_t stride,
              const float *table, int32_t table_size, int32_t trans,
              om_refmat *out) {
    memset(out, 0, sizeof(*out));
    if (table_size < 0 || table_size > MAX_STEP) return -1;   /* :25 */
    if (table_size == 0) return 0;                            /* :26 */

    out->table_size = table_size;
    out->table = (float *)malloc(sizeof(float) * (size_t)(table_size + 1));
    if (!out->table) return -1;
    memcpy(out->table, table, sizeof(float) * (size_t)table_size);   /* :29-31 */
    out->table[table_size] = 0.0f;

    const int32_t s_rows = trans ? cols : rows;   /* S-view shape */
    const int32_t s_cols = trans ? rows : cols;
    const uint8_t filler = (uint8_t)table_size;

    stream_t st = {0};
    panels_t pn = {0};
    for (int32_t c0 = 0; c0 < s_cols; c0 += PANEL_W) {
        const int32_t w = (s_cols - c0) < PANEL_W ? (s_cols - c0) : PANEL_W;
        const int64_t begin = st.n;
        int32_t prev = 0;
        for (int32_t r = 0; r < s_rows; r++) {
            for (int32_t c = 0; c < w; c++) {
                const int64_t src = trans ? (int64_t)(c0 + c) * stride + r
                                          : (int64_t)r * stride + (c0 + c);
                const uint8_t id = dm[src];
                if (id >= table_size) continue;
                if (emit_entry(&st, &prev, r * PANEL_W + c, id, filler)) goto oom;
            }
        }
        if (st.n != begin) {                                  /* :57-60 */
            if (panels_push(&pn, 0, c0, begin, st.n)) goto oom;
        }
    }
    out->rows = s_rows;                                       /* :63-64, :96-97 */
    out->cols = s_cols;
    out->n_entries = st.n;
    out->pos = st.pos;
    out->val = st.val;
    out->n_panels = pn.n;
    out->panel_row_off = pn.ro;
    out->panel_col_off = pn.co;
    out->panel_begin = pn.b;
    out->panel_end = pn.e;
    return 0;
oom:
    free(st.pos); free(st.val);
    free(pn.ro); free(pn.co); free(pn.b); free(pn.e);
    free(out->table);
    memset(out, 0, sizeof(*out));
    return -1;
}

void om_free(om_refmat *m) {
    free(m->table); free(m->pos); free(m->val);
    free(m->panel_row_off); free(m->panel_col_off);
    free(m->panel_begin); free(m->panel_end);
    memset(m, 0, sizeof(*m));
}

int64_t om_nnz(const om_refmat *m) {
    int64_t n = 0;
    for (int64_t e = 0; e < m->n_entries; e++) n += (m->val[e] < m->table_size);
    return n;
}

/* Walk one panel's delta stream; call `fn` for every stored entry with its
 * S-row, S-column and codebook id (decode of sparse-matrix.cc:116-121 and
 * kernel.cc:780-790: running prefix sum, row = off>>8, col = off&255). */
#define FOR_EACH_ENTRY(m, p, SROW, SCOL, ID, BODY)                              \
    do {                                                                        \
        int32_t off_ = 0;                                                       \
        for (int64_t e_ = (m)->panel_begin[p]; e_ < (m)->panel_end[p]; e_++) {  \
            off_ += (m)->pos[e_];                                               \
            if ((m)->val[e_] >= (m)->table_size) continue;                      \
            const int32_t SROW = (m)->panel_row_off[p] + (off_ >> PANEL_SHIFT); \
            const int32_t SCOL = (m)->panel_col_off[p] + (off_ & PANEL_MASK);   \
            const uint8_t ID = (m)->val[e_];                                    \
            BODY;                                                               \
        }                                                                       \
    } while (0)

/* CopyTo, sparse-matrix.cc:101-137. */
void om_decode_dense(const om_refmat *m, float *out, int32_t stride, int32_t trans) {
    const int64_t nrows_out = trans ? m->cols : m->rows;
    memset(out, 0, sizeof(float) * (size_t)(nrows_out * stride));
    for (int32_t p = 0; p < m->n_panels; p++) {
        FOR_EACH_ENTRY(m, p, r, c, id, {
            if (trans) out[(int64_t)c * stride + r] = m->table[id];
            else       out[(int64_t)r * stride + c] = m->table[id];
        });
    }
}

/* kernel.cc:10-29: c[i][j] *= beta over m x n. */
void om_beta(float *c, int32_t m, int32_t n, int32_t ldc, float beta) {
    for (int32_t i = 0; i < m; i++)
        for (int32_t j = 0; j < n; j++) c[(int64_t)i * ldc + j] *= beta;
}

/* kernel.cc:31-187: sa[j*ldsa + i] = a[i*lda + j]. */
void om_transpose(const float *a, int32_t m, int32_t n, int32_t lda, float *sa, int32_t ldsa) {
    for (int32_t i = 0; i < m; i++)
        for (int32_t j = 0; j < n; j++) sa[(int64_t)j * ldsa + i] = a[(int64_t)i * lda + j];
}

/* AddMatMat, sparse-matrix.cc:139-194.  C (m x n) = alpha*A(m x k)*S + beta*C.
 * The reference transposes A and C through scratch buffers (exact copies,
 * :180-189) and, per panel, walks the entries in stream order, applying
 * c[i][col] += a[i][row] * (table[id] * alpha) for every i (kernel.cc:791,
 * 568-582).  For a fixed output element the contributions therefore arrive
 * in ascending S-row order; we reproduce exactly that sequence of roundings. */
void om_addmatmat(const om_refmat *m, const float *a, int32_t mm, int32_t lda,
                  float *c, int32_t ldc, float alpha, float beta) {
    if (beta != 1.0f) om_beta(c, mm, m->cols, ldc, beta);      /* :149-151 */
    if (alpha == 0.0f) return;                                  /* :152 */
    for (int32_t p = 0; p < m->n_panels; p++) {
        FOR_EACH_ENTRY(m, p, r, col, id, {
            const float v = m->table[id] * alpha;               /* kernel.cc:791 */
            for (int32_t i = 0; i < mm; i++) {
                float *ci = &c[(int64_t)i * ldc + col];
                const float prod = a[(int64_t)i * lda + r] * v;
                *ci = *ci + prod;                               /* kernel.cc:569-582 */
            }
        });
    }
}

/* CSR of B = S^T: B row = S column, B column = S row. */
void om_to_csr(const om_refmat *m, int64_t *row_ptr, int32_t *col_idx,
               float *val, uint8_t *tid) {
    const int32_t n = m->cols;
    memset(row_ptr, 0, sizeof(int64_t) * (size_t)(n + 1));
    for (int32_t p = 0; p < m->n_panels; p++)
        FOR_EACH_ENTRY(m, p, r, c, id, { (void)r; (void)id; row_ptr[c + 1]++; });
    for (int32_t j = 0; j < n; j++) row_ptr[j + 1] += row_ptr[j];
    int64_t *fill = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    memcpy(fill, row_ptr, sizeof(int64_t) * (size_t)n);
    for (int32_t p = 0; p < m->n_panels; p++) {
        FOR_EACH_ENTRY(m, p, r, c, id, {
            const int64_t at = fill[c]++;
            col_idx[at] = r;
            if (val) val[at] = m->table[id];
            if (tid) tid[at] = id;
        });
    }
    free(fill);
}

#define CSR_SPMV_BODY(RP)                                                      \
    for (int64_t r = 0; r < n_rows; r++) {                                     \
        float acc = y[r];                                                      \
        if (beta != 1.0f) acc = acc * beta;                                    \
        if (alpha != 0.0f) {                                                   \
            for (int64_t e = RP[r]; e < RP[r + 1]; e++) {                      \
                const float v = val[e] * alpha;                                \
                const float prod = x[col_idx[e]] * v;                          \
                acc = acc + prod;                                              \
            }                                                                  \
        }                                                                      \
        y[r] = acc;                                                            \
    }

void om_csr_spmv(int64_t n_rows, const int64_t *row_ptr, const int32_t *col_idx,
                 const float *val, const float *x, float *y, float alpha, float beta) {
    CSR_SPMV_BODY(row_ptr)
}

void om_csr_spmv_i32(int64_t n_rows, const int32_t *row_ptr, const int32_t *col_idx,
                     const float *val, const float *x, float *y, float alpha, float beta) {
    CSR_SPMV_BODY(row_ptr)
}

/* The same kernel with the rows split over n_threads OpenMP threads (SURVEY §8d
 * baseline B2, "all cores"): every row is still summed by one thread in the
 * reference's order, so the result is bit-identical to om_csr_spmv_i32. */
void om_csr_spmv_i32_mt(int64_t n_rows, const int32_t *row_ptr, const int32_t *col_idx,
                        const float *val, const float *x, float *y, float alpha, float beta,
                        int32_t n_threads) {
#pragma omp parallel for schedule(static) num_threads(n_threads)
    for (int64_t r0 = 0; r0 < n_rows; r0 += 4096) {
        const int64_t r1 = r0 + 4096 < n_rows ? r0 + 4096 : n_rows;
        for (int64_t r = r0; r < r1; r++) {
            float acc = y[r];
            if (beta != 1.0f) acc = acc * beta;
            if (alpha != 0.0f) {
                for (int64_t e = row_ptr[r]; e < row_ptr[r + 1]; e++) {
                    const float v = val[e] * alpha;
                    const float prod = x[col_idx[e]] * v;
                    acc = acc + prod;
                }
            }
            y[r] = acc;
        }
    }
}

void om_csr_spmm(int64_t n_rows, const int64_t *row_ptr, const int32_t *col_idx,
                 const float *val, int32_t n_rhs, const float *X, int64_t ldx,
                 float *Y, int64_t ldy, float alpha, float beta) {
    for (int64_t r = 0; r < n_rows; r++) {
        float *yr = &Y[r * ldy];
        if (beta != 1.0f)
            for (int32_t j = 0; j < n_rhs; j++) yr[j] = yr[j] * beta;
        if (alpha == 0.0f) continue;
        for (int64_t e = row_ptr[r]; e < row_ptr[r + 1]; e++) {
            const float v = val[e] * alpha;
            const float *xr = &X[(int64_t)col_idx[e] * ldx];
            for (int32_t j = 0; j < n_rhs; j++) {
                const float prod = xr[j] * v;
                yr[j] = yr[j] + prod;
            }
        }
    }
}

/* NOT the reference: a model of SM_ALGO_MFMA's arithmetic (sparsematrix_amd/csrc/
 * spmm_mfma.hip), for its test only.  v_mfma_f32_16x16x4_f32 is an exact f32 fma chain in
 * k order (MI355X_MICROARCH.md), so each output is beta*y then fmaf(fl(v*alpha), x, acc)
 * over the row's terms in stored order -- one rounding per term where the reference
 * (om_csr_spmm above, kernel.cc:568-582) rounds the product and the sum separately. */
void om_csr_spmm_fma(int64_t n_rows, const int64_t *row_ptr, const int32_t *col_idx,
                     const float *val, int32_t n_rhs, const float *X, int64_t ldx,
                     float *Y, int64_t ldy, float alpha, float beta) {
    for (int64_t r = 0; r < n_rows; r++) {
        float *yr = &Y[r * ldy];
        if (beta != 1.0f)
            for (int32_t j = 0; j < n_rhs; j++) yr[j] = yr[j] * beta;
        if (alpha == 0.0f) continue;
        for (int64_t e = row_ptr[r]; e < row_ptr[r + 1]; e++) {
            const float v = val[e] * alpha;
            const float *xr = &X[(int64_t)col_idx[e] * ldx];
            for (int32_t j = 0; j < n_rhs; j++) yr[j] = fmaf(v, xr[j], yr[j]);
        }
    }
}

void om_csr_spmv_f64(int64_t n_rows, const int64_t *row_ptr, const int32_t *col_idx,
                     const float *val, const float *x, const float *y_in,
                     double *y, double *absum, float alpha, float beta) {
    for (int64_t r = 0; r < n_rows; r++) {
        double b = (double)y_in[r] * (beta != 1.0f ? (double)beta : 1.0);
        double acc = b, ab = b < 0 ? -b : b;
        if (alpha != 0.0f) {
            for (int64_t e = row_ptr[r]; e < row_ptr[r + 1]; e++) {
                const double t = (double)val[e] * (double)alpha * (double)x[col_idx[e]];
                acc += t;
                ab += t < 0 ? -t : t;
            }
        }
        y[r] = acc;
        absum[r] = ab;
    }
}
