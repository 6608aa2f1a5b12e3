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
