"""The multi-GPU context of the C ABI (sm_multi_*, sparsematrix_amd/csrc/multi.cpp).

CPU: the partition arithmetic against the Python restatement, and the argument /
no-device error paths.  GPU (one MI355X: nranks = 1, RCCL with a single rank): the
context's SpMV, SpMM, pipelined batch and bare all-gather give the local products
bit for bit.  Multi-rank correctness of partition + all-gather + local product is
covered with gloo in test_distributed_gloo.py (the data path there is the same
restated split; RCCL itself needs one GPU per rank)."""
import ctypes as C

import numpy as np
import pytest

import sparsematrix_amd as sm
from sparsematrix_amd import _lib
from sparsematrix_amd.distributed import MultiContext, RowPartition, partition_c


@pytest.mark.parametrize("n,world", [(10, 3), (1 << 26, 8), (7, 8), (0, 2), (1 << 20, 1),
                                     (999_999_937, 7)])
def test_partition_matches_restatement(n, world):
    bounds = [partition_c(n, world, r) for r in range(world)]
    assert bounds == [RowPartition(n, world).bounds(r) for r in range(world)]
    assert bounds[0][0] == 0 and bounds[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(bounds, bounds[1:]))
    sizes = [b - a for a, b in bounds]
    assert max(sizes) - min(sizes) <= 1


def test_partition_and_create_argument_errors():
    L = _lib.load()
    r0, r1 = C.c_int64(), C.c_int64()
    for args in ((-1, 2, 0), (10, 0, 0), (10, 2, 2), (10, 2, -1)):
        assert L.sm_multi_partition(*args, C.byref(r0), C.byref(r1)) == _lib.SM_ERR_INVALID_ARG
    out = C.c_void_p()
    uid = _lib.SmUniqueId()
    assert L.sm_multi_create(C.byref(uid), 2, 0, None, C.byref(out)) == _lib.SM_ERR_INVALID_ARG
    assert L.sm_multi_create(C.byref(uid), 2, 5, None, C.byref(out)) == _lib.SM_ERR_INVALID_ARG
    assert b"null" in L.sm_multi_last_error() or b"rank" in L.sm_multi_last_error()
    assert L.sm_multi_spmv(None, 1.0, None, 1.0, None, 0, None) == _lib.SM_ERR_INVALID_ARG


@pytest.mark.gpu
def test_multi_single_rank_equals_local():
    import torch
    import oracle
    oracle.build()
    sm.load()
    n_rows, n_cols = 50000, 60000
    rng = np.random.default_rng(7)
    cols = np.sort(rng.integers(0, n_cols, (n_rows, 12)), axis=1)
    ci = cols.reshape(-1).astype(np.int32)
    rp = np.arange(0, ci.size + 1, 12, dtype=np.int32)
    table = rng.uniform(-1, 1, 255).astype(np.float32)
    va = table[rng.integers(0, 255, ci.size)]
    M = sm.SparseMatrix.from_csr(rp, ci, va, n_cols)
    ctx = MultiContext(M, 1, 0, MultiContext.unique_id())
    dev = torch.device("cuda")
    xs = [torch.from_numpy(rng.uniform(-1, 1, n_cols).astype(np.float32)).to(dev) for _ in range(5)]
    y0 = torch.from_numpy(rng.uniform(-1, 1, n_rows).astype(np.float32)).to(dev)
    want = []
    for x in xs:
        y = y0.clone()
        M.spmv(x, y, 1.3, 0.7)
        want.append(y)
    # one product at a time, with timing
    ctx.set_timing(True)
    for x, w in zip(xs, want):
        y = y0.clone()
        ctx.spmv(x, y, 1.3, 0.7)
        torch.cuda.synchronize()
        assert torch.equal(y.view(torch.int32), w.view(torch.int32))
    ag, comp = ctx.last_times()
    assert ag >= 0.0 and comp > 0.0
    # pipelined batch: all-gathers on the context's stream beside the SpMVs
    ys = [y0.clone() for _ in xs]
    ctx.spmv_batch(xs, ys, 1.3, 0.7)
    torch.cuda.synchronize()
    for y, w in zip(ys, want):
        assert torch.equal(y.view(torch.int32), w.view(torch.int32))
    # bare all-gather: the gathered x is x itself at one rank
    p = ctx.allgather(xs[2])
    torch.cuda.synchronize()
    got = np.empty(n_cols, np.float32)
    torch.cuda.synchronize()
    from sparsematrix_amd.sparse_matrix import _ptr  # noqa: F401
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipMemcpy(ctypes.c_void_p(got.ctypes.data), ctypes.c_void_p(p),
                         ctypes.c_size_t(4 * n_cols), 2) == 0
    assert np.array_equal(got, xs[2].cpu().numpy())
    # SpMM through the context: the X panel gathered, then the row-panel kernel
    X = torch.from_numpy(rng.uniform(-1, 1, (n_cols, 32)).astype(np.float32)).to(dev)
    Y0 = torch.from_numpy(rng.uniform(-1, 1, (n_rows, 32)).astype(np.float32)).to(dev)
    Yw, Yg = Y0.clone(), Y0.clone()
    M.spmm(X, Yw, 1.3, 0.7)
    ctx.spmm(X, Yg, 1.3, 0.7)
    torch.cuda.synchronize()
    assert torch.equal(Yg.view(torch.int32), Yw.view(torch.int32))
    ctx.close()
