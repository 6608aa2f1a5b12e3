/*
 * oracle/refmodel.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of NeverLEX/sparsematrix's CPU algorithm for the
 * sparse x dense hot path (SparseMatrix<uint8,uint8,float>, panels of 256
 * columns, uint8 delta positions, uint8 codebook ids).  It is the checker the
 * HIP product is compared against; nothing under sparsematrix_amd/ links or
 * calls it.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may use it.
 *
 * Parity pin: the fixtures in tests/golden hold outputs of the real reference compiled
 * from /root/reference by oracle/Makefile (oracle/_ref/libsblas_ref.so, built
 * in the development container only).  tests/test_oracle_golden.py checks
 * this restatement bit-for-bit against every fixture.
 *
 * All arithmetic follows the reference's order exactly; build with
 * -ffp-contract=off so that `c += a * v` stays a separate multiply and add,
 * as in the reference's generic-C path (kernel.cc:568-582).
 */
#ifndef SM_ORACLE_REFMODEL_H
#define SM_ORACLE_REFMODEL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Encoded matrix in the reference's storage format (sparse-matrix.h:46-52).
 * rows/cols are the S view (rows_ = k, cols_ = n). */
typedef struct om_refmat {
    int32_t rows, cols;
    int32_t table_size;        /* valid table entries T; table[T] == 0 */
    float *table;              /* T + 1 floats */
    int64_t n_entries;         /* E = stored nonzeros + filler steps */
    uint8_t *pos;              /* E delta steps */
    uint8_t *val;              /* E codebook ids (T marks a filler) */
    int32_t n_panels;
    int32_t *panel_row_off, *panel_col_off;   /* block_bounds_ */
    int64_t *panel_begin, *panel_end;         /* block_index_bounds_ */
} om_refmat;

/* CopyForm: sparse-matrix.cc:20-99.  Returns 0 on success. */
int om_encode(const uint8_t *dm, int32_t rows, int32_t cols, int32_t stride,
              const float *table, int32_t table_size, int32_t trans,
              om_refmat *out);
void om_free(om_refmat *m);

/* CopyTo: sparse-matrix.cc:101-137. */
void om_decode_dense(const om_refmat *m, float *out, int32_t stride, int32_t trans);

/* AddMatMat: sparse-matrix.cc:139-194 (beta kernel.cc:10-29, decode
 * kernel.cc:771-800, axpy kernel.cc:568-582). a: m x k (lda), c: m x n (ldc). */
void om_addmatmat(const om_refmat *m, const float *a, int32_t mm, int32_t lda,
                  float *c, int32_t ldc, float alpha, float beta);

/* Number of stored (non-filler) entries. */
int64_t om_nnz(const om_refmat *m);

/* CSR of B = S^T (n rows, k cols), rows in ascending column order, i.e. the
 * per-output order the reference accumulates in.  tid (optional) receives the
 * codebook id per nonzero.  row_ptr has n+1 entries. */
void om_to_csr(const om_refmat *m, int64_t *row_ptr, int32_t *col_idx,
               float *val, uint8_t *tid);

/* Same-order CSR kernels (bit-exact with om_addmatmat for the matching m):
 *   y[r] = (beta != 1 ? beta*y[r] : y[r]); if alpha != 0:
 *   for e in row r (ascending): y[r] = y[r] + x[col[e]] * (val[e]*alpha)
 * SpMM: X is k x N row-major (ldx), Y is n x N row-major (ldy). */
void om_csr_spmv(int64_t n_rows, const int64_t *row_ptr, const int32_t *col_idx,
                 const float *val, const float *x, float *y, float alpha, float beta);
void om_csr_spmm(int64_t n_rows, const int64_t *row_ptr, const int32_t *col_idx,
                 const float *val, int32_t n_rhs, const float *X, int64_t ldx,
                 float *Y, int64_t ldy, float alpha, float beta);
/* Not the reference: the fma-chain model of SM_ALGO_MFMA (tests only). */
void om_csr_spmm_fma(int64_t n_rows, const int64_t *row_ptr, const int32_t *col_idx,
                 const float *val, int32_t n_rhs, const float *X, int64_t ldx,
                 float *Y, int64_t ldy, float alpha, float beta);

/* Same as om_csr_spmv but with int32 row_ptr (the device format). */
void om_csr_spmv_i32(int64_t n_rows, const int32_t *row_ptr, const int32_t *col_idx,
                     const float *val, const float *x, float *y, float alpha, float beta);
void om_csr_spmv_i32_mt(int64_t n_rows, const int32_t *row_ptr, const int32_t *col_idx,
                        const float *val, const float *x, float *y, float alpha, float beta,
                        int32_t n_threads);

/* fp64 reference and per-row sum of |terms| (for tolerance pins). */
void om_csr_spmv_f64(int64_t n_rows, const int64_t *row_ptr, const int32_t *col_idx,
                     const float *val, const float *x, const float *y_in,
                     double *y, double *absum, float alpha, float beta);

/* kernel.cc:10-29 and kernel.cc:31-187 (exact copies, any order). */
void om_beta(float *c, int32_t m, int32_t n, int32_t ldc, float beta);
void om_transpose(const float *a, int32_t m, int32_t n, int32_t lda, float *sa, int32_t ldsa);

#ifdef __cplusplus
}
#endif
#endif
