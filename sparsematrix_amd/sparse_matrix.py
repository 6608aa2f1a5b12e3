"""Host-side mirror of the reference operator surface, over the C ABI.

``SparseMatrix`` follows ``sblas::SparseMatrix<uint8, uint8, float>``
(reference src/sparse/sparse-matrix.h:25-53) name for name: ``CopyForm``,
``CopyTo``, ``AddMatMat``, ``NumRows``, ``NumCols``, ``Destroy``,
``operator==`` (``__eq__``) and ``SelfTest``.  Host (numpy) operands go through
the synchronous, bit-exact ``sm_addmatmat_host``; device (torch, ``cuda``)
operands go through the asynchronous device entry points on the current
stream.  The device-level calls the benchmarks use are ``spmv`` / ``spmm``.

All arithmetic happens in the HIP kernels of libsparsematrix_amd.so.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _lib
from ._lib import ALGOS, SM_NO_TRANS, SM_TRANS, SmInfo, check

SblasNoTrans = SM_NO_TRANS   # SBLAS_TRANSPOSE, sparse-matrix.h:20-23
SblasTrans = SM_TRANS


def _ptr(a) -> int:
    """Raw pointer of a numpy array or torch tensor (None -> 0)."""
    if a is None:
        return 0
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return int(a.data_ptr())


def _is_device(a) -> bool:
    return a is not None and not isinstance(a, np.ndarray) and getattr(a, "is_cuda", False)


def _stream_of(t, stream) -> int:
    if stream is not None:
        return int(stream) if isinstance(stream, int) else int(stream.cuda_stream)
    import torch
    return int(torch.cuda.current_stream(t.device).cuda_stream)


def _check_dev(t, min_elems: int, name: str) -> None:
    """Device operand guard: the C ABI takes raw pointers and cannot see sizes."""
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a CUDA (HIP) torch tensor")
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32")
    if t.numel() < min_elems:
        raise ValueError(f"{name} has {t.numel()} elements, needs at least {min_elems}")


def _check_dev_2d(t, rows: int, cols: int, name: str) -> None:
    _check_dev(t, 0, name)
    if t.dim() != 2 or (t.shape[1] > 1 and t.stride(1) != 1) or t.shape[0] < rows \
            or t.shape[1] < cols:
        raise ValueError(f"{name} must be a row-major {rows} x {cols} (or larger) view")


def _algo(algo) -> int:
    if isinstance(algo, int):
        return algo
    try:
        return ALGOS[algo]
    except KeyError:
        raise ValueError(f"algo must be one of {sorted(ALGOS)}") from None


class SparseMatrix:
    """sblas::SparseMatrix<uint8,uint8,float> on an MI355X (device-resident CSR of B = S^T)."""

    def __init__(self, density_matrix=None, rows: int = 0, cols: int = 0, stride: int = 0,
                 vals=None, val_table_size: int = 0, trans: int = SblasNoTrans,
                 device: int = 0):
        self._h = None
        self.device = device
        self._L = _lib.load()
        if density_matrix is not None:
            self.CopyForm(density_matrix, rows, cols, stride, vals, val_table_size, trans)

    # ---- lifetime ---------------------------------------------------------
    def Destroy(self) -> None:
        """sparse-matrix.cc:9-18."""
        if self._h:
            self._L.sm_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.Destroy()
        except Exception:
            pass

    def _require(self):
        if not self._h:
            raise RuntimeError("SparseMatrix is empty (call CopyForm or from_csr first)")
        return self._h

    def _dims(self):
        """(n_rows, n_cols) of the held matrix, cached per handle: the per-call operand
        guards of spmv/spmm then cost no sm_get_info round trip."""
        h = self._require()
        if getattr(self, "_dims_h", None) != h:
            inf = self.info()
            self._dims_cache = (inf["n_rows"], inf["n_cols"])
            self._dims_h = h
        return self._dims_cache

    # ---- construction -----------------------------------------------------
    def CopyForm(self, density_matrix, rows: int, cols: int, stride: int, vals,
                 val_table_size: int, trans: int = SblasNoTrans) -> None:
        """sparse-matrix.cc:20-99: encode a rows x stride uint8 id matrix with a float table."""
        dm = np.ascontiguousarray(density_matrix, dtype=np.uint8).reshape(-1)
        if dm.size < rows * stride and rows * cols > 0 and val_table_size > 0:
            raise ValueError("density_matrix smaller than rows * stride")
        tb = np.zeros(max(int(val_table_size), 1), np.float32)
        if val_table_size:
            tb[:val_table_size] = np.asarray(vals, np.float32).reshape(-1)[:val_table_size]
        h = C.c_void_p()
        st = self._L.sm_create_from_dense_index(_ptr(dm), rows, cols, stride, _ptr(tb),
                                                val_table_size, int(trans), self.device,
                                                C.byref(h))
        check(st, "CopyForm")
        self.Destroy()
        self._h = h

    @classmethod
    def from_dense_index(cls, index, rows: int, cols: int, stride: int, vals,
                         val_table_size: int, trans: int = SblasNoTrans, device: int = 0,
                         stream=None) -> "SparseMatrix":
        """CopyForm from a uint8 id matrix (rows x stride): a torch cuda tensor is scanned
        on the device (sm_create_from_dense_index_device), anything else on the host."""
        self = cls(device=device)
        if not _is_device(index):
            self.CopyForm(index, rows, cols, stride, vals, val_table_size, trans)
            return self
        import torch
        assert index.dtype == torch.uint8
        dm = index.contiguous()
        if dm.numel() < rows * stride and rows * cols > 0 and val_table_size > 0:
            raise ValueError("index smaller than rows * stride")
        tb = np.zeros(max(int(val_table_size), 1), np.float32)
        if val_table_size:
            tb[:val_table_size] = np.asarray(vals, np.float32).reshape(-1)[:val_table_size]
        h = C.c_void_p()
        st = self._L.sm_create_from_dense_index_device(_ptr(dm), rows, cols, stride, _ptr(tb),
                                                       val_table_size, int(trans), device,
                                                       _stream_of(dm, stream), C.byref(h))
        check(st, "from_dense_index")
        self._h = h
        return self

    @classmethod
    def from_csr(cls, row_ptr, col_idx, val, n_cols: int, device: int = 0,
                 stream=None, opts: Optional[dict] = None) -> "SparseMatrix":
        """Additive CSR ingestion of B (n_rows x n_cols): numpy (host) or torch cuda tensors.

        `opts` (optional) forces the SpMV layout, e.g. ``{"layout": "exact"}`` or
        ``{"layout": "cband", "band_slabs": 1}`` -- the fields of sm_build_opts."""
        self = cls(device=device)
        n_rows = int(row_ptr.shape[0]) - 1
        nnz = int(col_idx.shape[0])
        h = C.c_void_p()
        o = _lib.build_opts(**(opts or {}))
        if _is_device(row_ptr):
            import torch
            assert row_ptr.dtype == torch.int32 and col_idx.dtype == torch.int32
            assert val.dtype == torch.float32
            rp, ci, va = row_ptr.contiguous(), col_idx.contiguous(), val.contiguous()
            st = self._L.sm_create_from_csr_device_ex(n_rows, n_cols, nnz, _ptr(rp), _ptr(ci),
                                                      _ptr(va), device, _stream_of(rp, stream),
                                                      C.byref(o), C.byref(h))
        else:
            rp = np.ascontiguousarray(row_ptr, np.int32)
            ci = np.ascontiguousarray(col_idx, np.int32)
            va = np.ascontiguousarray(val, np.float32)
            st = self._L.sm_create_from_csr_ex(n_rows, n_cols, nnz, _ptr(rp), _ptr(ci), _ptr(va),
                                               device, C.byref(o), C.byref(h))
        check(st, "from_csr")
        self._h = h
        return self

    # ---- queries ----------------------------------------------------------
    def NumRows(self) -> int:
        """rows_ = k of the S view (sparse-matrix.h:39)."""
        return int(self._L.sm_num_rows(self._h)) if self._h else 0

    def NumCols(self) -> int:
        """cols_ = n of the S view (sparse-matrix.h:40)."""
        return int(self._L.sm_num_cols(self._h)) if self._h else 0

    def info(self) -> dict:
        inf = SmInfo()
        check(self._L.sm_get_info_ex(self._require(), C.byref(inf), C.sizeof(inf)), "sm_get_info")
        return {k: getattr(inf, k) for k, _ in SmInfo._fields_}

    def layout_digest(self) -> tuple:
        """sm_layout_digest: FNV-1a digests of the relabeling, the sliced ELL's structure, its
        slots and its codebook (0 where not built)."""
        d = (C.c_uint64 * 4)()
        check(self._L.sm_layout_digest(self._require(), d), "sm_layout_digest")
        return tuple(int(v) for v in d)

    @property
    def n_rows(self) -> int:
        return self.info()["n_rows"]

    @property
    def n_cols(self) -> int:
        return self.info()["n_cols"]

    @property
    def nnz(self) -> int:
        return self.info()["nnz"]

    def csr(self):
        """Host copy of the device CSR of B: (row_ptr, col_idx, val)."""
        inf = self.info()
        rp = np.zeros(inf["n_rows"] + 1, np.int32)
        ci = np.zeros(max(inf["nnz"], 1), np.int32)
        va = np.zeros(max(inf["nnz"], 1), np.float32)
        check(self._L.sm_copy_csr(self._h, _ptr(rp), _ptr(ci), _ptr(va)), "sm_copy_csr")
        return rp, ci[: inf["nnz"]], va[: inf["nnz"]]

    def build_ref_stream(self, table: Optional[np.ndarray] = None) -> None:
        """Encode a CSR-built matrix in the reference's format (sm_build_ref_stream,
        sparse-matrix.cc:20-99): afterwards ref_stream(), == and algo="native" serve it.
        `table`: the codebook (<= 255 fp32 values every value must match); None takes the
        values' distinct bit patterns in CSR order."""
        if table is None:
            check(self._L.sm_build_ref_stream(self._h, None, 0), "sm_build_ref_stream")
            return
        tb = np.ascontiguousarray(table, np.float32)
        check(self._L.sm_build_ref_stream(self._h, _ptr(tb), int(tb.size)), "sm_build_ref_stream")

    def ref_stream(self) -> dict:
        """The reference encoding (pos_index_, val_index_, block bounds)."""
        inf = self.info()
        E, P = inf["n_entries"], inf["n_panels"]
        pos = np.zeros(max(E, 1), np.uint8)
        val = np.zeros(max(E, 1), np.uint8)
        ro = np.zeros(max(P, 1), np.int32)
        co = np.zeros(max(P, 1), np.int32)
        b = np.zeros(max(P, 1), np.int64)
        e = np.zeros(max(P, 1), np.int64)
        check(self._L.sm_copy_ref_stream(self._h, _ptr(pos), _ptr(val), _ptr(ro), _ptr(co),
                                         _ptr(b), _ptr(e)), "sm_copy_ref_stream")
        return dict(rows=inf["s_rows"], cols=inf["s_cols"], pos=pos[:E], val=val[:E],
                    panel_row_off=ro[:P], panel_col_off=co[:P], panel_begin=b[:P],
                    panel_end=e[:P])

    def CopyTo(self, density_matrix: Optional[np.ndarray], stride: int,
               trans: int = SblasNoTrans) -> np.ndarray:
        """sparse-matrix.cc:101-137: decode into a dense float matrix (host)."""
        inf = self.info()
        nr = inf["s_cols"] if trans else inf["s_rows"]
        if density_matrix is None:
            density_matrix = np.zeros(max(nr * stride, 1), np.float32)
        out = density_matrix
        if not (isinstance(out, np.ndarray) and out.dtype == np.float32 and out.flags.c_contiguous):
            raise TypeError("CopyTo needs a C-contiguous float32 numpy array")
        if out.size < nr * stride:
            raise ValueError("output smaller than rows * stride")
        check(self._L.sm_to_dense(self._h, _ptr(out), stride, int(trans)), "CopyTo")
        return out

    def __eq__(self, other) -> bool:
        """operator== (sparse-matrix.cc:197-207)."""
        if not isinstance(other, SparseMatrix):
            return NotImplemented
        if not self._h or not other._h:
            return not self._h and not other._h
        return bool(self._L.sm_equal(self._h, other._h))

    __hash__ = None

    # ---- compute ------------------------------------------------------------
    def AddMatMat(self, a, m: int, lda: int, c, ldc: int, alpha: float, beta: float,
                  algo="parity", stream=None):
        """sparse-matrix.cc:139-194: C (m x n) = alpha * A (m x k) * S + beta * C, in place.

        numpy operands: synchronous and bit-identical to the reference.
        torch cuda operands: asynchronous on the current stream with `algo`."""
        h = self._require()
        k, n = self.NumRows(), self.NumCols()
        need_a = (m - 1) * lda + k if (m > 0 and alpha != 0.0 and k > 0) else 0
        need_c = (m - 1) * ldc + n if (m > 0 and n > 0) else 0
        if _is_device(c):
            _check_dev(c, need_c, "c")
            if need_a:
                _check_dev(a, need_a, "a")
            st = self._L.sm_addmatmat(h, _ptr(a), m, lda, _ptr(c), ldc, alpha, beta, _algo(algo),
                                      _stream_of(c, stream))
        else:
            if not (isinstance(c, np.ndarray) and c.dtype == np.float32 and c.flags.c_contiguous):
                raise TypeError("host AddMatMat needs C-contiguous float32 numpy arrays")
            a_arr = np.ascontiguousarray(a, np.float32)
            if c.size < need_c or a_arr.size < need_a:
                raise ValueError("a or c smaller than the (m, lda/ldc) layout requires")
            st = self._L.sm_addmatmat_host(h, _ptr(a_arr), m, lda, _ptr(c), ldc, alpha, beta)
        check(st, "AddMatMat")
        return c

    def spmv(self, x, y, alpha: float = 1.0, beta: float = 1.0, algo="auto", stream=None):
        """y = alpha * B * x + beta * y on device tensors (float32, contiguous)."""
        n_rows, n_cols = self._dims()
        _check_dev(x, n_cols, "x")
        _check_dev(y, n_rows, "y")
        if (x.dim() != 1 and not x.is_contiguous()) or (y.dim() != 1 and not y.is_contiguous()):
            raise ValueError("x and y must be contiguous")
        if x.dim() == 1 and x.stride(0) != 1 or y.dim() == 1 and y.stride(0) != 1:
            raise ValueError("x and y must be unit-stride")
        st = self._L.sm_spmv(self._require(), alpha, _ptr(x), beta, _ptr(y), _algo(algo),
                             _stream_of(y, stream))
        check(st, "sm_spmv")
        return y

    def spmm(self, X, Y, alpha: float = 1.0, beta: float = 1.0, algo="auto", stream=None):
        """Y (n x N) = alpha * B * X (k x N) + beta * Y, row-major device tensors."""
        n_rhs = int(Y.shape[1])
        n_rows, n_cols = self._dims()
        _check_dev_2d(X, n_cols, n_rhs, "X")
        _check_dev_2d(Y, n_rows, n_rhs, "Y")
        st = self._L.sm_spmm(self._require(), n_rhs, alpha, _ptr(X), int(X.stride(0)), beta,
                             _ptr(Y), int(Y.stride(0)), _algo(algo), _stream_of(Y, stream))
        check(st, "sm_spmm")
        return Y

    # ---- the reference's own known-answer test -------------------------------
    @staticmethod
    def SelfTest(device: int = 0, seed: int = 0) -> bool:
        """sparse-matrix.cc:209-313, run through this library: the two 3x2/2x3 KATs and
        a 1023 x 511 (stride 512) NoTrans/Trans round trip at 25 % density."""
        table8 = np.array([1.1, 2.2, 3.3, 4.4, 5.5, 6.6, 7.7, 8.8], np.float32)
        want = np.array([1.1, 0, 0, 4.4, 8.8, 0], np.float32)
        for dm, rows, cols, stride, trans in (
                (np.array([0, 255, 255, 3, 7, 255], np.uint8), 3, 2, 2, SblasNoTrans),
                (np.array([0, 255, 7, 255, 3, 255], np.uint8), 2, 3, 3, SblasTrans)):
            sm = SparseMatrix(dm, rows, cols, stride, table8, 8, trans, device=device)
            out = np.ones(6, np.float32)
            sm.CopyTo(out, 2)
            if not np.array_equal(out, want):
                return False
            if trans:
                out = np.ones(6, np.float32)
                sm.CopyTo(out, stride, SblasTrans)
                if not np.array_equal(out, np.array([1.1, 0, 8.8, 0, 4.4, 0], np.float32)):
                    return False
            a = np.array([3.1, 5, 7], np.float32)
            c = np.array([4, 8], np.float32)
            sm.AddMatMat(a, 1, 3, c, 2, 1.3, 2.0)
            if abs(c[0] - 92.513) > 1e-3 or abs(c[1] - 44.6) > 1e-3:
                return False
        rng = np.random.default_rng(seed)
        m, n, stride = 1023, 511, 512
        live = np.zeros(m * stride, bool)
        live[rng.permutation(m * stride)[: m * stride - int(m * stride * 0.75)]] = True
        table = rng.uniform(-1000, 1000, 64).astype(np.float32)
        index = np.where(live, rng.integers(0, 63, m * stride), 255).astype(np.uint8)
        matrix = np.where(live, table[np.minimum(index, 63)], 0).astype(np.float32)
        sm = SparseMatrix(device=device)
        for trans in (SblasNoTrans, SblasTrans):
            sm.CopyForm(index, m, n, stride, table, 63, trans)
            copy = np.zeros(m * stride, np.float32)
            sm.CopyTo(copy, stride, trans)
            if not np.array_equal(matrix.reshape(m, stride)[:, :n], copy.reshape(m, stride)[:, :n]):
                return False
        return True


# ---- kernel.h helpers on device tensors (kernel.cc:10-187) ---------------------------
def sblas_beta_operation_kernel(c, m: int, n: int, ldc: int, beta: float, stream=None):
    L = _lib.load()
    check(L.sm_beta_scale(_ptr(c), m, n, ldc, beta, _stream_of(c, stream)), "sm_beta_scale")
    return c


def sblas_trans_kernel(a, m: int, n: int, lda: int, sa, ldsa: int, stream=None):
    L = _lib.load()
    check(L.sm_transpose(_ptr(a), m, n, lda, _ptr(sa), ldsa, _stream_of(sa, stream)),
          "sm_transpose")
    return sa
