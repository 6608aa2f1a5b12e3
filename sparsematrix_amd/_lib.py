"""ctypes binding of the C ABI in include/sparsematrix.h.

The shared library is built in-tree (``make`` / ``__graft_entry__.build()``) as
``sparsematrix_amd/libsparsematrix_amd.so``.  There is no fallback: if the
library is missing or fails to load, every entry point raises.

HIP runtime note: PyTorch-ROCm ships its own ``libamdhip64.so`` (SONAME
``libamdhip64.so.7``).  When torch is importable it is imported *before* the
library is opened so that the already-loaded runtime satisfies the library's
``libamdhip64.so.7`` dependency and one process holds one HIP runtime.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# SM_LIB_PATH: development A/B of alternative builds of the same library (tools/).
LIB_PATH = os.environ.get("SM_LIB_PATH") or os.path.join(_HERE, "libsparsematrix_amd.so")

# sm_status
SM_OK = 0
SM_ERR_INVALID_ARG = 1
SM_ERR_OUT_OF_MEMORY = 2
SM_ERR_HIP = 3
SM_ERR_NOT_SUPPORTED = 4
SM_ERR_TOO_LARGE = 5
SM_ERR_INVALID_MATRIX = 6
SM_ERR_NO_DEVICE = 7

# sm_trans / sm_algo
SM_NO_TRANS, SM_TRANS = 0, 1
ALGOS = {"auto": 0, "parity": 1, "stream": 2, "vector": 3, "xband": 4, "sell": 5, "native": 6,
         "exact": 7, "mfma": 8, "merge": 9}

# Every symbol include/sparsematrix.h declares (tests check the .so exports them).
EXPORTS = (
    "sm_version", "sm_status_string", "sm_last_error", "sm_device_count",
    "sm_create_from_dense_index", "sm_create_from_dense_index_device", "sm_create_from_csr",
    "sm_create_from_csr_device", "sm_build_opts_init", "sm_create_from_csr_ex",
    "sm_create_from_csr_device_ex",
    "sm_destroy", "sm_get_info", "sm_get_info_ex", "sm_num_rows", "sm_num_cols", "sm_copy_ref_stream",
    "sm_build_ref_stream",
    "sm_copy_csr", "sm_to_dense", "sm_equal", "sm_spmv", "sm_spmm", "sm_addmatmat",
    "sm_addmatmat_host", "sm_beta_scale", "sm_transpose", "sm_panel_kernel", "sm_stream_sync",
    "sm_multi_last_error", "sm_multi_partition", "sm_multi_unique_id", "sm_multi_create",
    "sm_multi_destroy", "sm_multi_spmv", "sm_multi_spmm", "sm_multi_spmv_batch",
    "sm_multi_allgather", "sm_multi_set_timing", "sm_multi_last_times", "sm_multi_create_with",
    "sm_debug_seed_handoff", "sm_layout_digest",
)

SM_UNIQUE_ID_BYTES = 128


class SmUniqueId(C.Structure):
    _fields_ = [("internal", C.c_char * SM_UNIQUE_ID_BYTES)]


# sm_allgather_fn / sm_collective (include/sparsematrix.h): a caller-supplied all-gather.
SmAllgatherFn = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p)


class SmCollective(C.Structure):
    _fields_ = [("allgather", SmAllgatherFn), ("user", C.c_void_p)]


class SmInfo(C.Structure):
    _fields_ = [
        ("s_rows", C.c_int64), ("s_cols", C.c_int64), ("n_rows", C.c_int64),
        ("n_cols", C.c_int64), ("nnz", C.c_int64), ("table_size", C.c_int32),
        ("has_ref_stream", C.c_int32), ("n_entries", C.c_int64), ("n_panels", C.c_int64),
        ("device", C.c_int32), ("n_tiles", C.c_int32), ("n_long_rows", C.c_int32),
        ("max_row_nnz", C.c_int32), ("has_xband", C.c_int32), ("xband_blocks", C.c_int32),
        ("xband_bands", C.c_int32), ("xband_slabs", C.c_int32), ("xband_block_rows", C.c_int32),
        ("device_bytes", C.c_int64), ("col_relabel", C.c_int32), ("xband_slab_cols", C.c_int32),
        ("sell_slices", C.c_int64), ("sell_codebook", C.c_int32), ("ccsell_chunks", C.c_int32),
        ("hot_cols", C.c_int32), ("sweep_blocks", C.c_int32),
        ("exact_sell_slices", C.c_int64), ("exact_algo", C.c_int32), ("xband_slab0_cols", C.c_int32),
        ("merge_stage", C.c_int32), ("xband_beta_last", C.c_int32),
    ]


# sm_layout
LAYOUTS = {"auto": 0, "exact": 1, "blocked": 2, "gather": 3, "band2": 4, "cband": 5,
           "no_bands": 6, "bands": 7, "sweep": 8, "gcb": 9}


class SmBuildOpts(C.Structure):
    _fields_ = [
        ("struct_size", C.c_int32), ("layout", C.c_int32), ("band_slabs", C.c_int32),
        ("band_tall", C.c_int32), ("gather_band_log2", C.c_int32), ("sell", C.c_int32),
        ("sell_codebook", C.c_int32), ("sell_max_len", C.c_int32), ("sell_streams", C.c_int32),
        ("sell_sigma", C.c_int64), ("relabel", C.c_int32), ("tile_nnz", C.c_int32),
        ("ccsell", C.c_int32), ("ccsell_chunk_log2", C.c_int32), ("hot_cols", C.c_int32),
        ("exact_sell", C.c_int32), ("band_slab0_permille", C.c_int32), ("merge_stage", C.c_int32),
        ("host_build", C.c_int32),
    ]


def build_opts(**kw) -> SmBuildOpts:
    """sm_build_opts from keyword arguments (layout may be a name from LAYOUTS)."""
    o = SmBuildOpts()
    load().sm_build_opts_init(C.byref(o))
    for k, v in kw.items():
        if k == "layout" and isinstance(v, str):
            v = LAYOUTS[v]
        if k not in dict(SmBuildOpts._fields_):
            raise TypeError(f"unknown build option {k!r}")
        setattr(o, k, int(v))
    return o


class SparseMatrixError(RuntimeError):
    def __init__(self, status: int, where: str, message: str):
        self.status = status
        super().__init__(f"{where}: status {status}: {message}")


_lib = None
_lock = threading.Lock()

_vp, _i32, _i64, _f32 = C.c_void_p, C.c_int32, C.c_int64, C.c_float


def _declare(L):
    sig = {
        "sm_version": ([], C.c_char_p),
        "sm_status_string": ([C.c_int], C.c_char_p),
        "sm_last_error": ([], C.c_char_p),
        "sm_device_count": ([C.POINTER(_i32)], C.c_int),
        "sm_create_from_dense_index": ([_vp, _i32, _i32, _i32, _vp, _i32, C.c_int, _i32,
                                        C.POINTER(_vp)], C.c_int),
        "sm_create_from_dense_index_device": ([_vp, _i32, _i32, _i32, _vp, _i32, C.c_int, _i32,
                                               _vp, C.POINTER(_vp)], C.c_int),
        "sm_create_from_csr": ([_i64, _i64, _i64, _vp, _vp, _vp, _i32, C.POINTER(_vp)], C.c_int),
        "sm_create_from_csr_device": ([_i64, _i64, _i64, _vp, _vp, _vp, _i32, _vp,
                                       C.POINTER(_vp)], C.c_int),
        "sm_build_opts_init": ([C.POINTER(SmBuildOpts)], None),
        "sm_create_from_csr_ex": ([_i64, _i64, _i64, _vp, _vp, _vp, _i32, C.POINTER(SmBuildOpts),
                                   C.POINTER(_vp)], C.c_int),
        "sm_create_from_csr_device_ex": ([_i64, _i64, _i64, _vp, _vp, _vp, _i32, _vp,
                                          C.POINTER(SmBuildOpts), C.POINTER(_vp)], C.c_int),
        "sm_destroy": ([_vp], None),
        "sm_get_info": ([_vp, C.POINTER(SmInfo)], C.c_int),
        "sm_get_info_ex": ([_vp, C.POINTER(SmInfo), C.c_size_t], C.c_int),
        "sm_layout_digest": ([_vp, C.POINTER(C.c_uint64)], C.c_int),
        "sm_num_rows": ([_vp], _i32),
        "sm_num_cols": ([_vp], _i32),
        "sm_copy_ref_stream": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
        "sm_build_ref_stream": ([_vp, _vp, _i32], C.c_int),
        "sm_copy_csr": ([_vp, _vp, _vp, _vp], C.c_int),
        "sm_to_dense": ([_vp, _vp, _i32, C.c_int], C.c_int),
        "sm_equal": ([_vp, _vp], _i32),
        "sm_spmv": ([_vp, _f32, _vp, _f32, _vp, C.c_int, _vp], C.c_int),
        "sm_spmm": ([_vp, _i32, _f32, _vp, _i64, _f32, _vp, _i64, C.c_int, _vp], C.c_int),
        "sm_addmatmat": ([_vp, _vp, _i32, _i32, _vp, _i32, _f32, _f32, C.c_int, _vp], C.c_int),
        "sm_addmatmat_host": ([_vp, _vp, _i32, _i32, _vp, _i32, _f32, _f32], C.c_int),
        "sm_beta_scale": ([_vp, _i32, _i32, _i32, _f32, _vp], C.c_int),
        "sm_transpose": ([_vp, _i32, _i32, _i32, _vp, _i32, _vp], C.c_int),
        "sm_panel_kernel": ([_i32, _i32, _i32, _i32, _vp, _i32, _vp, _i32, _f32, _vp, _vp, _i32,
                             _vp, _i32, _vp], C.c_int),
        "sm_stream_sync": ([_vp], C.c_int),
        "sm_debug_seed_handoff": ([_vp, C.c_uint64], C.c_int),
        "sm_multi_last_error": ([], C.c_char_p),
        "sm_multi_partition": ([_i64, _i32, _i32, C.POINTER(_i64), C.POINTER(_i64)], C.c_int),
        "sm_multi_unique_id": ([C.POINTER(SmUniqueId)], C.c_int),
        "sm_multi_create": ([C.POINTER(SmUniqueId), _i32, _i32, _vp, C.POINTER(_vp)], C.c_int),
        "sm_multi_create_with": ([C.POINTER(SmCollective), _i32, _i32, _vp, C.POINTER(_vp)], C.c_int),
        "sm_multi_destroy": ([_vp], None),
        "sm_multi_spmv": ([_vp, _f32, _vp, _f32, _vp, C.c_int, _vp], C.c_int),
        "sm_multi_spmm": ([_vp, _i32, _f32, _vp, _f32, _vp, _i64, C.c_int, _vp], C.c_int),
        "sm_multi_spmv_batch": ([_vp, _i32, C.POINTER(_vp), _f32, C.POINTER(_vp), _f32,
                                 C.POINTER(_vp), C.c_int, _vp], C.c_int),
        "sm_multi_allgather": ([_vp, _vp, _i32, _vp, C.POINTER(_vp)], C.c_int),
        "sm_multi_set_timing": ([_vp, _i32], C.c_int),
        "sm_multi_last_times": ([_vp, C.POINTER(_f32), C.POINTER(_f32)], C.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res


def load(path: str | None = None):
    """Open the in-tree library (raises if it is missing: there is no fallback)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise ImportError(
                f"{p} not found: build it with `make` (or __graft_entry__.build()); "
                "sparsematrix_amd has no CPU fallback")
        try:  # one HIP runtime per process: let torch's libamdhip64 load first
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is part of this image
            pass
        L = C.CDLL(p, mode=C.RTLD_GLOBAL)
        _declare(L)
        _lib = L
        return L


def check(status: int, where: str) -> None:
    if status != SM_OK:
        L = load()
        raise SparseMatrixError(status, where, (L.sm_last_error() or b"").decode())


def check_multi(status: int, where: str) -> None:
    if status != SM_OK:
        L = load()
        raise SparseMatrixError(status, where, (L.sm_multi_last_error() or b"").decode())


def device_count() -> int:
    n = _i32(0)
    load().sm_device_count(C.byref(n))
    return int(n.value)
