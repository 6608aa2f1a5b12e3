// oracle/ref_capi.cc -- TEST INFRASTRUCTURE ONLY.
//
// A C-ABI wrapper around the REAL reference (NeverLEX/sparsematrix), compiled
// in place from /root/reference/src/sparse/{kernel.cc,sparse-matrix.cc} by
// oracle/Makefile into oracle/_ref/libsblas_ref.so.  It exists to pin the C
// restatement (oracle/refmodel.c) and to generate tests/golden/ fixtures
// (tools/gen_golden.py).  No reference source is copied into this repo; the
// reference's headers are included from /root/reference at build time.
//
// The encoded stream is private in the reference class (sparse-matrix.h:45-52);
// the checker needs it to pin bit-exact positions, so this translation unit
// (and only it) widens access before including the header.  Standard headers
// are included first so the macro only touches the reference class.
#include <cassert>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <utility>
#include <vector>
#include <unistd.h>

#define private public
#include "sparse-matrix.h"
#undef private

using Mat = sblas::SparseMatrix<uint8, uint8, float>;

extern "C" {

void *ref_create(const uint8_t *dm, int32_t rows, int32_t cols, int32_t stride,
                 const float *table, int32_t table_size, int32_t trans) {
    Mat *m = new Mat();
    m->rows_ = 0;
    m->cols_ = 0;
    m->CopyForm(dm, rows, cols, stride, table, table_size,
                trans ? sblas::SblasTrans : sblas::SblasNoTrans);
    return m;
}

void ref_destroy(void *h) { delete static_cast<Mat *>(h); }

int32_t ref_num_rows(void *h) { return static_cast<Mat *>(h)->NumRows(); }
int32_t ref_num_cols(void *h) { return static_cast<Mat *>(h)->NumCols(); }
int64_t ref_num_entries(void *h) { return (int64_t) static_cast<Mat *>(h)->pos_index_.size(); }
int32_t ref_num_panels(void *h) { return (int32_t) static_cast<Mat *>(h)->block_bounds_.size(); }
int32_t ref_table_size(void *h) { return (int32_t) static_cast<Mat *>(h)->val_table_.size() - 1; }

void ref_get_stream(void *h, uint8_t *pos, uint8_t *val) {
    Mat *m = static_cast<Mat *>(h);
    if (!m->pos_index_.empty()) memcpy(pos, m->pos_index_.data(), m->pos_index_.size());
    if (!m->val_index_.empty()) memcpy(val, m->val_index_.data(), m->val_index_.size());
}

void ref_get_panels(void *h, int32_t *row_off, int32_t *col_off, int32_t *begin, int32_t *end) {
    Mat *m = static_cast<Mat *>(h);
    for (size_t i = 0; i < m->block_bounds_.size(); i++) {
        row_off[i] = m->block_bounds_[i].first;
        col_off[i] = m->block_bounds_[i].second;
        begin[i] = m->block_index_bounds_[i].first;
        end[i] = m->block_index_bounds_[i].second;
    }
}

void ref_copyto(void *h, float *out, int32_t stride, int32_t trans) {
    static_cast<Mat *>(h)->CopyTo(out, stride, trans ? sblas::SblasTrans : sblas::SblasNoTrans);
}

void ref_addmatmat(void *h, float *a, int32_t m, int32_t lda, float *c, int32_t ldc,
                   float alpha, float beta) {
    static_cast<Mat *>(h)->AddMatMat(a, m, lda, c, ldc, alpha, beta);
}

int32_t ref_equal(void *h0, void *h1) { return *static_cast<Mat *>(h0) == *static_cast<Mat *>(h1); }

int32_t ref_selftest(void) {
    Mat m;
    return m.SelfTest() ? 1 : 0;
}

void ref_srand(uint32_t seed) { srand(seed); }

// kernel.h entry points (instantiated at kernel.cc:802-811).
void ref_beta(float *c, int m, int n, int ldc, float beta) {
    sblas_beta_operation_kernel<float>(c, m, n, ldc, beta);
}
void ref_trans(float *a, int m, int n, int lda, float *sa, int ldsa) {
    sblas_trans_kernel<float>(a, m, n, lda, sa, ldsa);
}
void ref_kernel_operation(int variant, int m, int n, int k, float *a, int lda, float *c, int ldc,
                          float alpha, uint8_t *ppos, uint8_t *pval, int pos_len,
                          float *table, int valid_table_size) {
    switch (variant) {
    case 0:
        sblas_kernel_operation<uint8_t, uint8_t, float, SBLAS_BLOCK_COL_SHIFT>(
            m, n, k, a, lda, c, ldc, alpha, ppos, pval, pos_len, table, valid_table_size);
        break;
    case 1:
        sblas_kernel_operation_naive<uint8_t, uint8_t, float, SBLAS_BLOCK_COL_SHIFT>(
            m, n, k, a, lda, c, ldc, alpha, ppos, pval, pos_len, table, valid_table_size);
        break;
    case 2:
        sblas_kernel_operation_trans<uint8_t, uint8_t, float, SBLAS_BLOCK_COL_SHIFT>(
            m, n, k, a, lda, c, ldc, alpha, ppos, pval, pos_len, table, valid_table_size);
        break;
    default:
        sblas_kernel_operation_trans_ex<uint8_t, uint8_t, float, SBLAS_BLOCK_COL_SHIFT>(
            m, n, k, a, lda, c, ldc, alpha, ppos, pval, pos_len, table, valid_table_size);
        break;
    }
}

}  // extern "C"
