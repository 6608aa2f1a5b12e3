"""oracle -- TEST INFRASTRUCTURE ONLY.

numpy/ctypes front end for the C restatement in ``oracle/refmodel.c`` (built to
``oracle/_build/liboracle.so``) and, in the development container only, for the
real reference compiled in place (``oracle/_ref/libsblas_ref.so``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg import this package, and only as the checker / the timed CPU baseline.  The
product (``sparsematrix_amd``) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_REF_PATH = os.path.join(_HERE, "_ref", "libsblas_ref.so")

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")


class _RefMat(C.Structure):
    _fields_ = [
        ("rows", C.c_int32), ("cols", C.c_int32), ("table_size", C.c_int32),
        ("table", C.POINTER(C.c_float)), ("n_entries", C.c_int64),
        ("pos", C.POINTER(C.c_uint8)), ("val", C.POINTER(C.c_uint8)),
        ("n_panels", C.c_int32),
        ("panel_row_off", C.POINTER(C.c_int32)), ("panel_col_off", C.POINTER(C.c_int32)),
        ("panel_begin", C.POINTER(C.c_int64)), ("panel_end", C.POINTER(C.c_int64)),
    ]


def build() -> None:
    """Compile the restatement (and the reference wrapper when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    if os.path.isdir("/root/reference/src/sparse"):
        subprocess.run(["make", "-s", "-C", _HERE, "ref"], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.om_encode.argtypes = [_u8p, C.c_int32, C.c_int32, C.c_int32, _f32p, C.c_int32,
                                C.c_int32, C.POINTER(_RefMat)]
        L.om_encode.restype = C.c_int
        L.om_free.argtypes = [C.POINTER(_RefMat)]
        L.om_decode_dense.argtypes = [C.POINTER(_RefMat), _f32p, C.c_int32, C.c_int32]
        L.om_addmatmat.argtypes = [C.POINTER(_RefMat), _f32p, C.c_int32, C.c_int32, _f32p,
                                   C.c_int32, C.c_float, C.c_float]
        L.om_nnz.argtypes = [C.POINTER(_RefMat)]
        L.om_nnz.restype = C.c_int64
        L.om_to_csr.argtypes = [C.POINTER(_RefMat), _i64p, _i32p, _f32p, _u8p]
        L.om_csr_spmv.argtypes = [C.c_int64, _i64p, _i32p, _f32p, _f32p, _f32p, C.c_float, C.c_float]
        L.om_csr_spmv_i32.argtypes = [C.c_int64, _i32p, _i32p, _f32p, _f32p, _f32p, C.c_float,
                                      C.c_float]
        L.om_csr_spmv_i32_mt.argtypes = [C.c_int64, _i32p, _i32p, _f32p, _f32p, _f32p, C.c_float,
                                         C.c_float, C.c_int32]
        L.om_csr_spmm.argtypes = [C.c_int64, _i64p, _i32p, _f32p, C.c_int32, _f32p, C.c_int64,
                                  _f32p, C.c_int64, C.c_float, C.c_float]
        L.om_csr_spmm_fma.argtypes = [C.c_int64, _i64p, _i32p, _f32p, C.c_int32, _f32p, C.c_int64,
                                  _f32p, C.c_int64, C.c_float, C.c_float]
        L.om_csr_spmv_f64.argtypes = [C.c_int64, _i64p, _i32p, _f32p, _f32p, _f32p, _f64p, _f64p,
                                      C.c_float, C.c_float]
        L.om_beta.argtypes = [_f32p, C.c_int32, C.c_int32, C.c_int32, C.c_float]
        L.om_transpose.argtypes = [_f32p, C.c_int32, C.c_int32, C.c_int32, _f32p, C.c_int32]
        _lib = L
    return _lib


@dataclass
class RefStream:
    """The reference's encoded members (sparse-matrix.h:46-52)."""
    rows: int
    cols: int
    table: np.ndarray          # T+1 floats, last is 0
    pos: np.ndarray            # uint8 deltas
    val: np.ndarray            # uint8 ids
    panel_row_off: np.ndarray
    panel_col_off: np.ndarray
    panel_begin: np.ndarray
    panel_end: np.ndarray


class RefModel:
    """CPU restatement of sblas::SparseMatrix<uint8,uint8,float> (CopyForm/CopyTo/AddMatMat)."""

    def __init__(self, dm: np.ndarray, rows: int, cols: int, stride: int, table: np.ndarray,
                 table_size: int, trans: bool = False):
        L = lib()
        self._m = _RefMat()
        dm = np.ascontiguousarray(dm, dtype=np.uint8).reshape(-1)
        tb = np.zeros(max(table_size, 1), np.float32)
        tb[:table_size] = np.asarray(table, np.float32).reshape(-1)[:table_size]
        rc = L.om_encode(dm, rows, cols, stride, tb, table_size, int(bool(trans)), C.byref(self._m))
        if rc != 0:
            raise MemoryError("om_encode failed")

    def __del__(self):
        if getattr(self, "_m", None) is not None and _lib is not None:
            _lib.om_free(C.byref(self._m))
            self._m = None

    @property
    def rows(self) -> int:
        return self._m.rows

    @property
    def cols(self) -> int:
        return self._m.cols

    def stream(self) -> RefStream:
        m = self._m
        E, P, T = m.n_entries, m.n_panels, m.table_size

        def arr(ptr, n, dt):
            if n == 0 or not ptr:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt, copy=True)

        return RefStream(m.rows, m.cols, arr(m.table, T + 1 if T else 0, np.float32),
                         arr(m.pos, E, np.uint8), arr(m.val, E, np.uint8),
                         arr(m.panel_row_off, P, np.int32), arr(m.panel_col_off, P, np.int32),
                         arr(m.panel_begin, P, np.int64), arr(m.panel_end, P, np.int64))

    def nnz(self) -> int:
        return int(lib().om_nnz(C.byref(self._m)))

    def copy_to(self, stride: int, trans: bool = False) -> np.ndarray:
        nr = self.cols if trans else self.rows
        out = np.empty(max(nr * stride, 1), np.float32)
        lib().om_decode_dense(C.byref(self._m), out, stride, int(bool(trans)))
        return out[: nr * stride]

    def add_mat_mat(self, a: np.ndarray, m: int, lda: int, c: np.ndarray, ldc: int,
                    alpha: float, beta: float) -> np.ndarray:
        a = np.ascontiguousarray(a, np.float32).reshape(-1)
        out = np.array(c, np.float32, copy=True).reshape(-1)
        if a.size == 0:
            a = np.zeros(1, np.float32)
        if out.size == 0:
            out = np.zeros(1, np.float32)
            lib().om_addmatmat(C.byref(self._m), a, m, lda, out, ldc, alpha, beta)
            return out[:0]
        lib().om_addmatmat(C.byref(self._m), a, m, lda, out, ldc, alpha, beta)
        return out

    def to_csr(self):
        """CSR of B = S^T: (row_ptr int64 [n+1], col_idx int32, val float32, tid uint8)."""
        n, nnz = self.cols, self.nnz()
        rp = np.zeros(n + 1, np.int64)
        ci = np.zeros(max(nnz, 1), np.int32)
        va = np.zeros(max(nnz, 1), np.float32)
        td = np.zeros(max(nnz, 1), np.uint8)
        lib().om_to_csr(C.byref(self._m), rp, ci, va, td)
        return rp, ci[:nnz], va[:nnz], td[:nnz]


def _nz1(a, dt):
    a = np.ascontiguousarray(a, dt).reshape(-1)
    return a if a.size else np.zeros(1, dt)


def csr_spmv(row_ptr, col_idx, val, x, y, alpha=1.0, beta=1.0) -> np.ndarray:
    """Same-order CSR SpMV: y = alpha*B*x + beta*y with the reference's rounding sequence."""
    row_ptr = np.ascontiguousarray(row_ptr)
    out = np.array(y, np.float32, copy=True).reshape(-1)
    n = row_ptr.shape[0] - 1
    if n == 0:
        return out
    if row_ptr.dtype == np.int32:
        lib().om_csr_spmv_i32(n, row_ptr, _nz1(col_idx, np.int32), _nz1(val, np.float32),
                              _nz1(x, np.float32), out, alpha, beta)
    else:
        lib().om_csr_spmv(n, row_ptr.astype(np.int64), _nz1(col_idx, np.int32),
                          _nz1(val, np.float32), _nz1(x, np.float32), out, alpha, beta)
    return out


def csr_spmv_mt(row_ptr, col_idx, val, x, y, alpha=1.0, beta=1.0, threads=1) -> np.ndarray:
    """csr_spmv with the rows split over `threads` OpenMP threads (int32 row_ptr);
    bit-identical to csr_spmv (each row is still summed in order by one thread)."""
    row_ptr = np.ascontiguousarray(row_ptr, np.int32)
    out = np.array(y, np.float32, copy=True).reshape(-1)
    n = row_ptr.shape[0] - 1
    if n > 0:
        lib().om_csr_spmv_i32_mt(n, row_ptr, _nz1(col_idx, np.int32), _nz1(val, np.float32),
                                 _nz1(x, np.float32), out, alpha, beta, int(threads))
    return out


def csr_spmm(row_ptr, col_idx, val, X, Y, alpha=1.0, beta=1.0) -> np.ndarray:
    """Same-order CSR SpMM: Y (n x N) = alpha*B*X + beta*Y, X k x N row-major."""
    X = np.ascontiguousarray(X, np.float32)
    out = np.array(Y, np.float32, copy=True)
    n, N = out.shape
    if n == 0 or N == 0:
        return out
    lib().om_csr_spmm(n, np.ascontiguousarray(row_ptr, np.int64), _nz1(col_idx, np.int32),
                      _nz1(val, np.float32), N, _nz1(X, np.float32), N, out.reshape(-1),
                      N, alpha, beta)
    return out


def csr_spmm_fma(row_ptr, col_idx, val, X, Y, alpha=1.0, beta=1.0) -> np.ndarray:
    """NOT the reference: the fma-chain model of SM_ALGO_MFMA (refmodel.c om_csr_spmm_fma)."""
    X = np.ascontiguousarray(X, np.float32)
    out = np.array(Y, np.float32, copy=True)
    n, N = out.shape
    if n == 0 or N == 0:
        return out
    lib().om_csr_spmm_fma(n, np.ascontiguousarray(row_ptr, np.int64), _nz1(col_idx, np.int32),
                          _nz1(val, np.float32), N, X, X.shape[1], out, N, alpha, beta)
    return out


def csr_spmv_f64(row_ptr, col_idx, val, x, y, alpha=1.0, beta=1.0):
    """fp64 result and per-row sum of |terms| (|beta*y| + sum |alpha*v*x|)."""
    row_ptr = np.ascontiguousarray(row_ptr, np.int64)
    n = row_ptr.shape[0] - 1
    yo = np.zeros(max(n, 1), np.float64)
    ab = np.zeros(max(n, 1), np.float64)
    lib().om_csr_spmv_f64(n, row_ptr, _nz1(col_idx, np.int32), _nz1(val, np.float32),
                          _nz1(x, np.float32), _nz1(y, np.float32), yo, ab, alpha, beta)
    return yo[:n], ab[:n]


def beta_scale(c: np.ndarray, m: int, n: int, ldc: int, beta: float) -> np.ndarray:
    out = np.array(c, np.float32, copy=True).reshape(-1)
    lib().om_beta(out, m, n, ldc, beta)
    return out


def transpose(a: np.ndarray, m: int, n: int, lda: int, ldsa: int, out_size: int) -> np.ndarray:
    sa = np.zeros(out_size, np.float32)
    lib().om_transpose(np.ascontiguousarray(a, np.float32).reshape(-1), m, n, lda, sa, ldsa)
    return sa


def ref_available() -> bool:
    return os.path.exists(_REF_PATH)


def ref_lib():
    """The real reference (dev container only). Raises if it was not built."""
    if not ref_available():
        raise FileNotFoundError(_REF_PATH)
    L = C.CDLL(_REF_PATH)
    L.ref_create.argtypes = [_u8p, C.c_int32, C.c_int32, C.c_int32, _f32p, C.c_int32, C.c_int32]
    L.ref_create.restype = C.c_void_p
    L.ref_destroy.argtypes = [C.c_void_p]
    for nm in ("ref_num_rows", "ref_num_cols", "ref_num_panels", "ref_table_size"):
        getattr(L, nm).argtypes = [C.c_void_p]
        getattr(L, nm).restype = C.c_int32
    L.ref_num_entries.argtypes = [C.c_void_p]
    L.ref_num_entries.restype = C.c_int64
    L.ref_get_stream.argtypes = [C.c_void_p, _u8p, _u8p]
    L.ref_get_panels.argtypes = [C.c_void_p, _i32p, _i32p, _i32p, _i32p]
    L.ref_copyto.argtypes = [C.c_void_p, _f32p, C.c_int32, C.c_int32]
    L.ref_addmatmat.argtypes = [C.c_void_p, _f32p, C.c_int32, C.c_int32, _f32p, C.c_int32,
                                C.c_float, C.c_float]
    L.ref_equal.argtypes = [C.c_void_p, C.c_void_p]
    L.ref_equal.restype = C.c_int32
    L.ref_selftest.restype = C.c_int32
    L.ref_srand.argtypes = [C.c_uint32]
    L.ref_beta.argtypes = [_f32p, C.c_int, C.c_int, C.c_int, C.c_float]
    L.ref_trans.argtypes = [_f32p, C.c_int, C.c_int, C.c_int, _f32p, C.c_int]
    L.ref_kernel_operation.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, _f32p, C.c_int, _f32p,
                                       C.c_int, C.c_float, _u8p, _u8p, C.c_int, _f32p, C.c_int]
    return L


class Reference:
    """Thin handle on the compiled reference's SparseMatrix (dev container only)."""

    def __init__(self, dm, rows, cols, stride, table, table_size, trans=False):
        self.L = ref_lib()
        dm = np.ascontiguousarray(dm, np.uint8).reshape(-1)
        tb = np.zeros(max(table_size, 1), np.float32)
        tb[:table_size] = np.asarray(table, np.float32).reshape(-1)[:table_size]
        self.h = self.L.ref_create(dm, rows, cols, stride, tb, table_size, int(bool(trans)))

    def __del__(self):
        if getattr(self, "h", None):
            self.L.ref_destroy(self.h)
            self.h = None

    @property
    def rows(self):
        return self.L.ref_num_rows(self.h)

    @property
    def cols(self):
        return self.L.ref_num_cols(self.h)

    def stream(self) -> RefStream:
        L, h = self.L, self.h
        E, P = L.ref_num_entries(h), L.ref_num_panels(h)
        pos = np.zeros(max(E, 1), np.uint8)
        val = np.zeros(max(E, 1), np.uint8)
        L.ref_get_stream(h, pos, val)
        ro, co, b, e = (np.zeros(max(P, 1), np.int32) for _ in range(4))
        L.ref_get_panels(h, ro, co, b, e)
        T = L.ref_table_size(h)
        return RefStream(self.rows, self.cols, np.zeros(0, np.float32), pos[:E], val[:E],
                         ro[:P], co[:P], b[:P].astype(np.int64), e[:P].astype(np.int64))

    def copy_to(self, stride, trans=False):
        nr = self.cols if trans else self.rows
        out = np.full(max(nr * stride, 1), np.nan, np.float32)
        self.L.ref_copyto(self.h, out, stride, int(bool(trans)))
        return out[: nr * stride]

    def add_mat_mat(self, a, m, lda, c, ldc, alpha, beta):
        a = np.array(a, np.float32, copy=True).reshape(-1)
        out = np.array(c, np.float32, copy=True).reshape(-1)
        if a.size == 0:
            a = np.zeros(1, np.float32)
        if out.size == 0:
            out = np.zeros(1, np.float32)
        self.L.ref_addmatmat(self.h, a, m, lda, out, ldc, alpha, beta)
        return out[: np.asarray(c).size]
