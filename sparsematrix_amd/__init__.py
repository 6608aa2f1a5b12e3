"""sparsematrix_amd -- MI355X-native sparse x dense multiply (SpMV / SpMM).

Drop-in for NeverLEX/sparsematrix's ``SparseMatrix::AddMatMat`` hot path:
hand-written HIP kernels for gfx950 behind a C ABI (include/sparsematrix.h),
a C++ shim with the reference's exact class/kernel signatures
(include/sblas/), and this Python mirror of the operator surface.
"""
from ._lib import ALGOS, SparseMatrixError, device_count, load  # noqa: F401
from .sparse_matrix import (SblasNoTrans, SblasTrans, SparseMatrix,  # noqa: F401
                            sblas_beta_operation_kernel, sblas_trans_kernel)

__all__ = ["SparseMatrix", "SblasNoTrans", "SblasTrans", "SparseMatrixError", "ALGOS",
           "device_count", "load", "sblas_beta_operation_kernel", "sblas_trans_kernel"]
