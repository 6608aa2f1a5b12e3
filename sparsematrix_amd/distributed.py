"""Row-partitioned multi-GPU SpMV: one process per GPU, one all-gather of x.

SURVEY.md §8(e): the rows of B (the outputs) are split into p equal contiguous
slices, one per rank; every rank keeps global column indices; x is split the
same way.  Per product the only exchange is one all-gather of x (RCCL over
xGMI via torch.distributed's "nccl" backend, or gloo on CPU for tests),
followed by the local SpMV into the rank's slice of y.  No other collective.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable


@dataclass(frozen=True)
class RowPartition:
    n_rows: int
    world: int

    def bounds(self, rank: int) -> tuple[int, int]:
        """[r0, r1) of `rank`: equal slices, the first n_rows % world ranks one row longer."""
        q, r = divmod(self.n_rows, self.world)
        r0 = rank * q + min(rank, r)
        return r0, r0 + q + (1 if rank < r else 0)

    def equal(self) -> bool:
        """all_gather_into_tensor needs equal counts per rank."""
        return self.n_rows % self.world == 0


def slice_csr(row_ptr, col_idx, val, r0: int, r1: int):
    """Rows [r0, r1) of a CSR (numpy or torch); columns stay global."""
    a, b = int(row_ptr[r0]), int(row_ptr[r1])
    rp = row_ptr[r0:r1 + 1] - row_ptr[r0]
    return rp, col_idx[a:b], val[a:b]


def allgather_spmv(local_spmv: Callable, x_local, x_full, y_local, group=None):
    """x_full <- all_gather(x_local); y_local <- local_spmv(x_full, y_local).

    `local_spmv(x_full, y_local)` is the rank's product (the HIP kernel through
    the C ABI on GPU ranks)."""
    import torch.distributed as dist
    dist.all_gather_into_tensor(x_full, x_local, group=group)
    return local_spmv(x_full, y_local)


def _same_buffer(a, b) -> bool:
    """True when two tensors/arrays overlap in memory (same storage start)."""
    pa = a.data_ptr() if hasattr(a, "data_ptr") else a.__array_interface__["data"][0]
    pb = b.data_ptr() if hasattr(b, "data_ptr") else b.__array_interface__["data"][0]
    na = a.numel() * a.element_size() if hasattr(a, "numel") else a.nbytes
    nb = b.numel() * b.element_size() if hasattr(b, "numel") else b.nbytes
    return pa < pb + nb and pb < pa + na


def allgather_spmv_pipelined(products, group=None):
    """A sequence of independent products, each `(local_spmv, x_local, x_full,
    y_local)`: the all-gather of product k+1 is in flight while product k's SpMV
    runs -- still one all-gather per product and no other collective.

    Ordering (GPU ranks, RCCL): the all-gather of k+1 is issued after the wait on
    all-gather k and before SpMV k is enqueued, so RCCL's stream waits for what the
    compute stream holds at that point (SpMV k-1) and then runs beside SpMV k;
    x_full of k+1 may therefore be the buffer SpMV k-1 read, never one still
    being read.  On gloo (CPU) the waits are blocking and the order is the plain
    one.  Returns the number of products."""
    import torch.distributed as dist
    it = iter(products)
    nxt = next(it, None)
    if nxt is None:
        return 0
    work = dist.all_gather_into_tensor(nxt[2], nxt[1], group=group, async_op=True)
    n = 0
    while nxt is not None:
        cur, cur_work = nxt, work
        cur_work.wait()
        nxt = next(it, None)
        if nxt is not None:
            if _same_buffer(nxt[2], cur[2]):
                raise ValueError("allgather_spmv_pipelined: consecutive products share one "
                                 "x_full buffer; the all-gather of product k+1 would overwrite "
                                 "x while SpMV k reads it (rotate at least two x_full buffers)")
            work = dist.all_gather_into_tensor(nxt[2], nxt[1], group=group, async_op=True)
        cur[0](cur[2], cur[3])
        n += 1
    return n


def partition_c(n_rows: int, world: int, rank: int) -> tuple[int, int]:
    """The C ABI's equal split (sm_multi_partition); RowPartition.bounds restates it."""
    import ctypes as C
    from . import _lib
    r0, r1 = C.c_int64(), C.c_int64()
    _lib.check_multi(_lib.load().sm_multi_partition(n_rows, world, rank, C.byref(r0), C.byref(r1)),
                     "sm_multi_partition")
    return int(r0.value), int(r1.value)


def host_staged_allgather(group=None):
    """An all-gather for `MultiContext.with_collective` (sm_multi_create_with): the
    rank's slice is copied to the host, gathered over `group` (any torch.distributed
    backend -- gloo for a CPU control plane), and the gathered vector copied back.  It
    synchronises the stream it is given and blocks until `recv` holds the result, as
    the C ABI allows.  For ranks RCCL cannot serve (two ranks on one GPU) and for tests;
    RCCL (MultiContext) is the production path."""
    import ctypes as C

    import torch
    import torch.distributed as dist
    hip = C.CDLL("libamdhip64.so")
    hip.hipStreamSynchronize.argtypes = [C.c_void_p]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    world = dist.get_world_size(group)

    def allgather(send, recv, count, stream, user):
        try:
            if hip.hipStreamSynchronize(stream) != 0:
                return 2
            mine = torch.empty(count, dtype=torch.float32)
            if count and hip.hipMemcpy(mine.data_ptr(), send, 4 * count, 2) != 0:   # D2H
                return 3
            full = torch.empty(count * world, dtype=torch.float32)
            dist.all_gather_into_tensor(full, mine, group=group)
            if count and hip.hipMemcpy(recv, full.data_ptr(), 4 * count * world, 1) != 0:   # H2D
                return 4
            return 0
        except Exception:  # noqa: BLE001 -- reported to the C side as a failure
            return 1
    return allgather


class MultiContext:
    """The C ABI's multi-GPU context (sm_multi_*, include/sparsematrix.h): one RCCL
    communicator over the ranks, one ncclAllGather of x per product, then the local
    SpMV.  `local` is this rank's rows of B with global columns (a SparseMatrix);
    `unique_id` the 128 bytes rank 0 made with MultiContext.unique_id() and handed to
    every rank (bench.py broadcasts it over torch.distributed's gloo group).
    `MultiContext.with_collective` builds the same context over a Python all-gather
    instead of RCCL (sm_multi_create_with)."""

    def __init__(self, local, nranks: int, rank: int, unique_id: bytes | None = None,
                 collective=None):
        import ctypes as C
        from . import _lib
        self._L = _lib.load()
        self.local = local                       # the context refers to it: keep it alive
        h = C.c_void_p()
        if collective is not None:
            self._cb = _lib.SmAllgatherFn(collective)   # keep the trampoline alive
            self._coll = _lib.SmCollective(self._cb, None)
            _lib.check_multi(self._L.sm_multi_create_with(C.byref(self._coll), nranks, rank,
                                                          local._require(), C.byref(h)),
                             "sm_multi_create_with")
        else:
            uid = _lib.SmUniqueId()
            C.memmove(C.addressof(uid), bytes(unique_id), _lib.SM_UNIQUE_ID_BYTES)
            _lib.check_multi(self._L.sm_multi_create(C.byref(uid), nranks, rank, local._require(),
                                                     C.byref(h)), "sm_multi_create")
        self._h = h
        self.nranks, self.rank = nranks, rank
        info = local.info()
        self.n_cols = int(info["n_cols"])
        self.n_rows = int(info["n_rows"])
        self.x_local_len = self.n_cols // nranks
        self.device = int(info["device"])

    @classmethod
    def with_collective(cls, local, nranks: int, rank: int, allgather):
        """The context over `allgather(send_ptr, recv_ptr, count, stream, user) -> int`
        (e.g. host_staged_allgather(group)) instead of RCCL."""
        return cls(local, nranks, rank, collective=allgather)

    def _check(self, t, length: int, what: str, rows: int | None = None):
        """The C side cannot check device buffers: dtype, layout, device and length."""
        import torch
        assert t.dtype == torch.float32, f"{what}: float32 expected, got {t.dtype}"
        assert t.is_cuda and t.device.index == self.device, \
            f"{what}: must be on cuda:{self.device}, got {t.device}"
        if rows is None:
            assert t.is_contiguous() and t.dim() == 1 and t.numel() == length, \
                f"{what}: contiguous vector of {length} floats expected, got {tuple(t.shape)}"
        else:
            assert t.dim() == 2 and t.shape[0] == length and t.shape[1] == rows, \
                f"{what}: ({length}, {rows}) expected, got {tuple(t.shape)}"

    @staticmethod
    def unique_id() -> bytes:
        import ctypes as C
        from . import _lib
        uid = _lib.SmUniqueId()
        _lib.check_multi(_lib.load().sm_multi_unique_id(C.byref(uid)), "sm_multi_unique_id")
        return C.string_at(C.addressof(uid), _lib.SM_UNIQUE_ID_BYTES)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.sm_multi_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _stream(t, stream) -> int:
        if stream is not None:
            return int(stream) if isinstance(stream, int) else int(stream.cuda_stream)
        import torch
        return int(torch.cuda.current_stream(t.device).cuda_stream)

    def spmv(self, x_local, y_local, alpha=1.0, beta=1.0, algo="auto", stream=None):
        from . import _lib
        from .sparse_matrix import _algo
        self._check(x_local, self.x_local_len, "x_local")
        self._check(y_local, self.n_rows, "y_local")
        _lib.check_multi(self._L.sm_multi_spmv(self._h, alpha, x_local.data_ptr(), beta,
                                               y_local.data_ptr(), _algo(algo),
                                               self._stream(y_local, stream)), "sm_multi_spmv")
        return y_local

    def spmm(self, X_local, Y_local, alpha=1.0, beta=1.0, algo="auto", stream=None):
        from . import _lib
        from .sparse_matrix import _algo
        n_rhs = int(Y_local.shape[1])
        self._check(X_local, self.x_local_len, "X_local", rows=n_rhs)
        assert X_local.is_contiguous(), "X_local: contiguous rows expected"
        self._check(Y_local, self.n_rows, "Y_local", rows=n_rhs)
        assert Y_local.stride(1) == 1, "Y_local: rows must be contiguous"
        _lib.check_multi(self._L.sm_multi_spmm(self._h, n_rhs, alpha, X_local.data_ptr(), beta,
                                               Y_local.data_ptr(), int(Y_local.stride(0)),
                                               _algo(algo), self._stream(Y_local, stream)),
                         "sm_multi_spmm")
        return Y_local

    def spmv_batch(self, xs, ys, alpha=1.0, beta=1.0, algo="auto", stream=None, mats=None):
        """Independent products ys[i] = alpha * B_i * allgather(xs[i]) + beta * ys[i],
        B_i = mats[i] (default: the context's matrix); all-gather i+1 beside SpMV i."""
        import ctypes as C
        from . import _lib
        from .sparse_matrix import _algo
        n = len(xs)
        assert len(ys) == n and (mats is None or len(mats) == n), "one x, y (and matrix) per product"
        for i in range(n):
            self._check(xs[i], self.x_local_len, f"xs[{i}]")
            rows = self.n_rows if mats is None else int(mats[i].info()["n_rows"])
            assert ys[i].dtype.is_floating_point and ys[i].numel() == rows and ys[i].is_contiguous(), \
                f"ys[{i}]: contiguous vector of {rows} floats expected"
            self._check(ys[i], rows, f"ys[{i}]")
        xa = (C.c_void_p * n)(*[x.data_ptr() for x in xs])
        ya = (C.c_void_p * n)(*[y.data_ptr() for y in ys])
        ma = (C.c_void_p * n)(*[m._require().value for m in mats]) if mats is not None else None
        _lib.check_multi(self._L.sm_multi_spmv_batch(self._h, n, ma, alpha, xa, beta, ya,
                                                     _algo(algo), self._stream(ys[0], stream)),
                         "sm_multi_spmv_batch")

    def allgather(self, x_local, n_rhs: int = 1, stream=None) -> int:
        import ctypes as C
        from . import _lib
        self._check(x_local.reshape(-1), self.x_local_len * n_rhs, "x_local")
        p = C.c_void_p()
        _lib.check_multi(self._L.sm_multi_allgather(self._h, x_local.data_ptr(), n_rhs,
                                                    self._stream(x_local, stream), C.byref(p)),
                         "sm_multi_allgather")
        return int(p.value or 0)

    def set_timing(self, on: bool) -> None:
        from . import _lib
        _lib.check_multi(self._L.sm_multi_set_timing(self._h, 1 if on else 0), "sm_multi_set_timing")

    def last_times(self) -> tuple[float, float]:
        import ctypes as C
        from . import _lib
        a, b = C.c_float(), C.c_float()
        _lib.check_multi(self._L.sm_multi_last_times(self._h, C.byref(a), C.byref(b)),
                         "sm_multi_last_times")
        return float(a.value), float(b.value)
