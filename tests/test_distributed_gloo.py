"""World-size-2 (and 3) CPU rehearsal of the multi-GPU path over gloo.

Each rank holds its equal row slice of B with global columns and its slice of
x; one all-gather of x, then the rank's local product.  On GPU ranks the local
product is the HIP kernel; here the oracle's same-order CSR SpMV stands in as
the local operator so that the partitioning, the all-gather and the slice
bookkeeping are checked bit-for-bit against the single-process oracle.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from sparsematrix_amd.distributed import RowPartition, allgather_spmv, slice_csr


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(n, per_row, seed):
    rng = np.random.default_rng(seed)
    cols = np.sort(rng.integers(0, n, (n, per_row)), axis=1).astype(np.int32)
    rp = np.arange(0, n * per_row + 1, per_row, dtype=np.int64)
    val = rng.uniform(-1, 1, n * per_row).astype(np.float32)
    x = rng.uniform(-1, 1, n).astype(np.float32)
    y = rng.uniform(-1, 1, n).astype(np.float32)
    return rp, cols.reshape(-1), val, x, y


def _worker(rank, world, port, n, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rp, ci, va, x, y = _problem(n, 16, seed=5)
    part = RowPartition(n, world)
    r0, r1 = part.bounds(rank)
    lrp, lci, lva = slice_csr(rp, ci, va, r0, r1)
    x_local = torch.from_numpy(x[r0:r1].copy())
    x_full = torch.empty(n, dtype=torch.float32)
    y_local = y[r0:r1].copy()

    def local(xf, yl):
        return oracle.csr_spmv(lrp, lci, lva, xf.numpy(), yl, 1.3, 0.7)

    out = allgather_spmv(local, x_local, x_full, y_local)
    assert np.array_equal(x_full.numpy(), x)
    gathered = [torch.empty(r1 - r0, dtype=torch.float32) for _ in range(world)]
    dist.all_gather(gathered, torch.from_numpy(out))
    if rank == 0:
        out_q.put(np.concatenate([g.numpy() for g in gathered]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_partition_allgather_matches_single_process(world):
    oracle.build()
    n = 3000 * world
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rp, ci, va, x, y = _problem(n, 16, seed=5)
    want = oracle.csr_spmv(rp, ci, va, x, y, 1.3, 0.7)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_partition_bounds():
    for n, w in ((10, 3), (8, 8), (1 << 20, 8), (7, 2)):
        p = RowPartition(n, w)
        b = [p.bounds(r) for r in range(w)]
        assert b[0][0] == 0 and b[-1][1] == n
        assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
        assert max(e - s for s, e in b) - min(e - s for s, e in b) <= 1
        assert p.equal() == (n % w == 0)


def _worker_pipelined(rank, world, port, n, n_prod, out_q):
    from sparsematrix_amd.distributed import allgather_spmv_pipelined
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rp, ci, va, _, y = _problem(n, 16, seed=9)
    part = RowPartition(n, world)
    r0, r1 = part.bounds(rank)
    lrp, lci, lva = slice_csr(rp, ci, va, r0, r1)
    xs = [np.random.default_rng(100 + k).uniform(-1, 1, n).astype(np.float32)
          for k in range(n_prod)]
    # two x_full buffers rotated as in bench.py: product k+1 gathers into the one product k-1 read
    bufs = [torch.empty(n, dtype=torch.float32) for _ in range(2)]
    outs = [None] * n_prod

    def product(k):
        def local(xf, yl):
            assert np.array_equal(xf.numpy(), xs[k])
            outs[k] = oracle.csr_spmv(lrp, lci, lva, xf.numpy(), yl, 1.0, 0.5)
        return (local, torch.from_numpy(xs[k][r0:r1].copy()), bufs[k % 2], y[r0:r1].copy())

    assert allgather_spmv_pipelined(product(k) for k in range(n_prod)) == n_prod
    res = []
    for k in range(n_prod):
        gathered = [torch.empty(r1 - r0, dtype=torch.float32) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(outs[k]))
        res.append(np.concatenate([g.numpy() for g in gathered]))
    if rank == 0:
        out_q.put(np.stack(res))
    dist.barrier()
    dist.destroy_process_group()


def test_pipelined_allgather_matches_single_process():
    """Independent products with the all-gather of k+1 issued before SpMV k:
    every product equals the single-process oracle bit-for-bit."""
    oracle.build()
    world, n, n_prod = 2, 4000, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_pipelined, args=(r, world, port, n, n_prod, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rp, ci, va, _, y = _problem(n, 16, seed=9)
    for k in range(n_prod):
        x = np.random.default_rng(100 + k).uniform(-1, 1, n).astype(np.float32)
        want = oracle.csr_spmv(rp, ci, va, x, y, 1.0, 0.5)
        assert np.array_equal(got[k].view(np.uint32), want.view(np.uint32)), k
