// include/sblas/sparse-matrix.h -- drop-in replacement for the reference's
// src/sparse/sparse-matrix.h (sparse-matrix.h:11-53).  Same typedefs, enum,
// class template, constructors and member functions; the matrix itself lives on
// the MI355X behind the C ABI (include/sparsematrix.h) and AddMatMat runs the
// gfx950 kernels (bit-identical to the reference on host operands).
// Only <uint8, uint8, float> is instantiated, as in the reference
// (sparse-matrix.cc:315).  Link with -lsblas -lsparsematrix_amd.
#ifndef SBLAS_AMD_SPARSE_MATRIX_H
#define SBLAS_AMD_SPARSE_MATRIX_H
#pragma once

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <iostream>
#include <vector>

#include "kernel.h"

typedef int8_t int8;
typedef int16_t int16;
typedef int32_t int32;
typedef uint8_t uint8;
typedef uint16_t uint16;
typedef uint32_t uint32;

struct sm_matrix;   // include/sparsematrix.h

namespace sblas {

enum SBLAS_TRANSPOSE { SblasNoTrans = 0, SblasTrans = 1 };

template <typename PosIndex_t, typename ValIndex_t, typename Value_t,
          const int32 block_row_shift = SBLAS_BLOCK_ROW_SHIFT,
          const int32 block_col_shift = SBLAS_BLOCK_COL_SHIFT>
class SparseMatrix {
public:
    SparseMatrix() {}
    SparseMatrix(const ValIndex_t *density_matrix, int32 rows, int32 cols, int32 stride,
                 const Value_t *vals, int32 val_table_size, SBLAS_TRANSPOSE trans = SblasNoTrans) {
        CopyForm(density_matrix, rows, cols, stride, vals, val_table_size, trans);
    }
    ~SparseMatrix() { Destroy(); }

    void Destroy();
    void CopyForm(const ValIndex_t *density_matrix, int32 rows, int32 cols, int32 stride,
                  const Value_t *vals, int32 val_table_size, SBLAS_TRANSPOSE trans = SblasNoTrans);
    void CopyTo(Value_t *density_matrix, int32 stride, SBLAS_TRANSPOSE trans = SblasNoTrans);
    void AddMatMat(Value_t *a, int32 m, int32 lda, Value_t *c, int32 ldc, Value_t alpha,
                   Value_t beta);

    int32 NumRows() const { return rows_; }
    int32 NumCols() const { return cols_; }

    bool operator==(const SparseMatrix<PosIndex_t, ValIndex_t, Value_t, block_row_shift,
                                       block_col_shift> &oth);
    bool SelfTest();

    // MI355X handle (for callers that also use the C ABI directly).
    sm_matrix *handle() const { return handle_; }

private:
    SparseMatrix(const SparseMatrix &) = delete;
    SparseMatrix &operator=(const SparseMatrix &) = delete;
    sm_matrix *handle_ = nullptr;
    int32 rows_ = 0;
    int32 cols_ = 0;
};

}  // namespace sblas

#endif
