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


def test_rccl_load_failure_reports_not_supported():
    """a failed dlopen of RCCL must come back as SM_ERR_NOT_SUPPORTED with the
    loader's message (it used to read dlerror() twice and crash on the NULL)."""
    import os
    import subprocess
    import sys
    code = ("import ctypes as C, sys; sys.path.insert(0, %r)\n"
            "from sparsematrix_amd import _lib\n"
            "L = _lib.load(); uid = _lib.SmUniqueId()\n"
            "st = L.sm_multi_unique_id(C.byref(uid))\n"
            "print(st, L.sm_multi_last_error().decode())\n") % os.path.dirname(os.path.dirname(__file__))
    env = dict(os.environ, SM_RCCL_LIB="/nonexistent/librccl-missing.so")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    st, msg = out.stdout.strip().split(" ", 1)
    assert int(st) == _lib.SM_ERR_NOT_SUPPORTED
    assert "cannot load librccl" in msg and "librccl-missing" in msg


def test_create_with_argument_errors():
    L = _lib.load()
    out = C.c_void_p()
    assert L.sm_multi_create_with(None, 2, 0, None, C.byref(out)) == _lib.SM_ERR_INVALID_ARG
    coll = _lib.SmCollective(_lib.SmAllgatherFn(lambda *a: 0), None)
    assert L.sm_multi_create_with(C.byref(coll), 2, 0, None, C.byref(out)) == _lib.SM_ERR_INVALID_ARG
    assert L.sm_multi_create_with(C.byref(coll), 0, 0, None, C.byref(out)) == _lib.SM_ERR_INVALID_ARG
    assert not out.value


def _small_problem(n_rows, n_cols, per, seed):
    rng = np.random.default_rng(seed)
    w = n_cols // per   # one column per stratum: distinct and sorted
    cols = np.arange(per)[None, :] * w + rng.integers(0, w, (n_rows, per))
    ci = cols.reshape(-1).astype(np.int32)
    rp = np.arange(0, ci.size + 1, per, dtype=np.int32)
    table = rng.uniform(-1, 1, 255).astype(np.float32)
    va = table[rng.integers(0, 255, ci.size)]
    return rp, ci, va


@pytest.mark.gpu
def test_multi_two_streams_single_rank():
    """products on one context from two streams take turns on the gather
    buffer -- every result equals the local product bit for bit."""
    import torch
    sm.load()
    n_rows, n_cols = 200000, 262144
    rp, ci, va = _small_problem(n_rows, n_cols, 16, 11)
    M = sm.SparseMatrix.from_csr(rp, ci, va, n_cols)
    ctx = MultiContext(M, 1, 0, MultiContext.unique_id())
    dev = torch.device("cuda")
    rng = np.random.default_rng(12)
    xs = [torch.from_numpy(rng.uniform(-1, 1, n_cols).astype(np.float32)).to(dev) for _ in range(6)]
    y0 = torch.from_numpy(rng.uniform(-1, 1, n_rows).astype(np.float32)).to(dev)
    want = []
    for x in xs:
        y = y0.clone()
        M.spmv(x, y, 1.0, 0.5)
        want.append(y)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    ys = [y0.clone() for _ in xs]
    torch.cuda.synchronize()
    for i, x in enumerate(xs):   # alternate streams, no host sync in between
        ctx.spmv(x, ys[i], 1.0, 0.5, stream=streams[i % 2])
    # and a batch on one stream right behind a single product on the other
    yb = [y0.clone() for _ in xs]
    torch.cuda.synchronize()
    ctx.spmv(xs[0], ys[0], 1.0, 0.5, stream=streams[0])
    ctx.spmv_batch(xs, yb, 1.0, 0.5, stream=streams[1])
    torch.cuda.synchronize()
    for i in range(len(xs)):
        assert torch.equal(yb[i].view(torch.int32), want[i].view(torch.int32)), i
        if i > 0:
            assert torch.equal(ys[i].view(torch.int32), want[i].view(torch.int32)), i
    ctx.close()


def _collective_worker(rank, world, port, out_q):
    import os
    import torch
    import torch.distributed as dist
    from sparsematrix_amd.distributed import host_staged_allgather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n_rows, n_cols = 24000, 48000
        rp, ci, va = _small_problem(n_rows, n_cols, 12, 21)
        part = RowPartition(n_rows, world)
        r0, r1 = part.bounds(rank)
        lrp = rp[r0:r1 + 1] - rp[r0]
        lci, lva = ci[rp[r0]:rp[r1]], va[rp[r0]:rp[r1]]
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        M = sm.SparseMatrix.from_csr(lrp.astype(np.int32), lci, lva, n_cols)
        ctx = MultiContext.with_collective(M, world, rank, host_staged_allgather())
        L = n_cols // world
        rng = np.random.default_rng(22)
        xs = [rng.uniform(-1, 1, n_cols).astype(np.float32) for _ in range(5)]
        y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
        xl = [torch.from_numpy(x[rank * L:(rank + 1) * L].copy()).to(dev) for x in xs]
        ys = [torch.from_numpy(y0[r0:r1].copy()).to(dev) for _ in xs]
        ctx.spmv_batch(xl, ys, 1.3, 0.7, algo="sell")          # pipelined C-ABI batch
        y1 = torch.from_numpy(y0[r0:r1].copy()).to(dev)
        ctx.spmv(xl[3], y1, 1.3, 0.7, algo="sell")              # one product
        X = np.random.default_rng(23).uniform(-1, 1, (n_cols, 8)).astype(np.float32)
        Y0 = np.random.default_rng(24).uniform(-1, 1, (n_rows, 8)).astype(np.float32)
        Yl = torch.from_numpy(Y0[r0:r1].copy()).to(dev)
        ctx.spmm(torch.from_numpy(X[rank * L:(rank + 1) * L].copy()).to(dev), Yl, 1.3, 0.7)
        torch.cuda.synchronize()
        res = [y.cpu() for y in ys] + [y1.cpu(), Yl.cpu().reshape(-1)]
        gathered = []
        for t in res:
            parts = [torch.empty(0)] * world
            dist.all_gather_object(parts, t)
            gathered.append(torch.cat(parts).numpy())
        if rank == 0:
            out_q.put(gathered)
        ctx.close()
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.gpu
def test_multi_collective_two_ranks_equals_single_process_oracle():
    """two ranks (one GPU, RCCL cannot serve that) drive the C-ABI
    multi path -- sm_multi_spmv_batch, sm_multi_spmv, sm_multi_spmm -- through a
    host-staged gloo all-gather (sm_multi_create_with); every output equals the
    single-process oracle bit for bit."""
    import socket
    import oracle
    import torch.multiprocessing as mp
    oracle.build()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_collective_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=110)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n_rows, n_cols = 24000, 48000
    rp, ci, va = _small_problem(n_rows, n_cols, 12, 21)
    rng = np.random.default_rng(22)
    xs = [rng.uniform(-1, 1, n_cols).astype(np.float32) for _ in range(5)]
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    for k in range(5):
        want = oracle.csr_spmv(rp, ci, va, xs[k], y0.copy(), 1.3, 0.7)
        assert np.array_equal(got[k].view(np.uint32), want.view(np.uint32)), k
    want = oracle.csr_spmv(rp, ci, va, xs[3], y0.copy(), 1.3, 0.7)
    assert np.array_equal(got[5].view(np.uint32), want.view(np.uint32))
    X = np.random.default_rng(23).uniform(-1, 1, (n_cols, 8)).astype(np.float32)
    Y0 = np.random.default_rng(24).uniform(-1, 1, (n_rows, 8)).astype(np.float32)
    Yw = oracle.csr_spmm(rp, ci, va, X, Y0.copy(), 1.3, 0.7)
    assert np.array_equal(got[6].view(np.uint32), Yw.reshape(-1).view(np.uint32))
