// include/sblas/kernel.h -- drop-in replacement for the reference's
// src/sparse/kernel.h (kernel.h:22-62): same macros, same template entry
// points, implemented by libsblas.so on top of the C ABI (sparsematrix.h), so
// every call runs on the MI355X.
//
// Pointers may be host or device memory: host operands are staged through the
// device and copied back (synchronous, like the reference); device operands are
// used in place on the default stream.  Instantiated for float (and the
// <uint8_t, uint8_t, float, 8> panel kernels), as the reference is
// (kernel.cc:802-811).
#ifndef SBLAS_AMD_KERNEL_H
#define SBLAS_AMD_KERNEL_H
#pragma once

#include <cassert>
#include <iostream>
#include <stdlib.h>
#include <unistd.h>

#define SBLAS_ASSERT assert
#define SBLAS_MALLOC malloc
#define SBLAS_FREE free
#define SBLAS_BLOCK_ROW_SHIFT 0
#define SBLAS_BLOCK_COL_SHIFT 8
#define SBLAS_MEMALIGN(align, size, pp_orig) \
    (!posix_memalign(pp_orig, align, size) ? *(pp_orig) : NULL)
#define SBLAS_MEMALIGN_FREE(x) \
    if (x) free(x), x = NULL;

// c[i*ldc + j] *= beta, i < m, j < n                      (kernel.cc:10-29)
template <typename type_t>
void sblas_beta_operation_kernel(type_t *c, int m, int n, int ldc, type_t beta);

// sa[j*ldsa + i] = a[i*lda + j], i < m, j < n              (kernel.cc:31-187)
template <typename type_t>
void sblas_trans_kernel(type_t *a, int m, int n, int lda, type_t *sa, int ldsa);

// One panel of the reference stream applied to C += A * S_panel * alpha.
// operation / _naive: A m x k (lda), C m x n (ldc)        (kernel.cc:213-338)
// _trans / _trans_ex: A^T k x (lda), C^T n x (ldc)       (kernel.cc:340-369, 771-800)
template <typename PosIndex_t, typename ValIndex_t, typename Value_t, const int block_col_shift>
void sblas_kernel_operation(int m, int n, int k, Value_t *a, int lda, Value_t *c, int ldc,
                            Value_t alpha, PosIndex_t *ppos, ValIndex_t *pval, int pos_len,
                            Value_t *val_table, int valid_table_size);

template <typename PosIndex_t, typename ValIndex_t, typename Value_t, const int block_col_shift>
void sblas_kernel_operation_naive(int m, int n, int k, Value_t *a, int lda, Value_t *c, int ldc,
                                  Value_t alpha, PosIndex_t *ppos, ValIndex_t *pval, int pos_len,
                                  Value_t *val_table, int valid_table_size);

template <typename PosIndex_t, typename ValIndex_t, typename Value_t, const int block_col_shift>
void sblas_kernel_operation_trans(int m, int n, int k, Value_t *a, int lda, Value_t *c, int ldc,
                                  Value_t alpha, PosIndex_t *ppos, ValIndex_t *pval, int pos_len,
                                  Value_t *val_table, int valid_table_size);

template <typename PosIndex_t, typename ValIndex_t, typename Value_t, const int block_col_shift>
void sblas_kernel_operation_trans_ex(int m, int n, int k, Value_t *a, int lda, Value_t *c,
                                     int ldc, Value_t alpha, PosIndex_t *ppos, ValIndex_t *pval,
                                     int pos_len, Value_t *val_table, int valid_table_size);

#endif
