"""Shared helpers for the -m gpu parity tests (device buffers via torch)."""
from __future__ import annotations

import numpy as np

TOL = 1e-6   # north_star: "within 1e-6 relative" -- defined against sum |terms|


def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    return torch


def to_dev(a: np.ndarray):
    torch = torch_dev()
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def to_host(t) -> np.ndarray:
    torch = torch_dev()
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def assert_terms_close(got: np.ndarray, want: np.ndarray, absum: np.ndarray, tol: float = TOL):
    """|got - want| <= tol * sum|terms| elementwise (and NaN where want is NaN)."""
    got = np.asarray(got, np.float64).reshape(-1)
    want = np.asarray(want, np.float64).reshape(-1)
    absum = np.asarray(absum, np.float64).reshape(-1)
    nan_w = np.isnan(want)
    assert np.array_equal(nan_w, np.isnan(got)), "NaN pattern differs"
    ok = ~nan_w
    err = np.abs(got[ok] - want[ok])
    bound = tol * absum[ok] + 1e-37
    bad = err > bound
    assert not bad.any(), (f"{int(bad.sum())} elements out of bound; worst ratio "
                           f"{float((err / bound).max()):.3g}")


def bits(a) -> np.ndarray:
    return np.ascontiguousarray(a, np.float32).reshape(-1).view(np.uint32)


def uniform_csr(n_rows: int, n_cols: int, per_row: int, seed: int, table=None):
    """`per_row` distinct sorted columns per row, values from a 255-entry table."""
    rng = np.random.default_rng(seed)
    cols = np.sort(rng.integers(0, n_cols, (n_rows, per_row), dtype=np.int64), axis=1)
    # make columns distinct within a row: bump duplicates forward, then re-sort
    for _ in range(8):
        dup = np.zeros_like(cols, bool)
        dup[:, 1:] = cols[:, 1:] == cols[:, :-1]
        if not dup.any():
            break
        cols[dup] = rng.integers(0, n_cols, int(dup.sum()))
        cols.sort(axis=1)
    if table is None:
        table = rng.uniform(-1, 1, 255).astype(np.float32)
    val = table[rng.integers(0, len(table), n_rows * per_row)].astype(np.float32)
    rp = np.arange(0, n_rows * per_row + 1, per_row, dtype=np.int32)
    return rp, cols.reshape(-1).astype(np.int32), val


def skewed_csr(n_rows: int, n_cols: int, lengths: np.ndarray, seed: int):
    """CSR with the given row lengths (unsorted columns allowed to repeat)."""
    rng = np.random.default_rng(seed)
    lengths = np.asarray(lengths, np.int64)
    rp = np.zeros(n_rows + 1, np.int64)
    rp[1:] = np.cumsum(lengths)
    nnz = int(rp[-1])
    col = np.empty(nnz, np.int32)
    for r in range(n_rows):
        col[rp[r]:rp[r + 1]] = np.sort(rng.integers(0, n_cols, int(lengths[r])))
    val = rng.uniform(-1, 1, nnz).astype(np.float32)
    return rp.astype(np.int32), col, val


def with_env(key: str, value: str, fn):
    """Run fn() with os.environ[key] = value (restored afterwards)."""
    import os
    old = os.environ.get(key)
    os.environ[key] = value
    try:
        return fn()
    finally:
        if old is None:
            os.environ.pop(key, None)
        else:
            os.environ[key] = old


def slab_order_spmv(rp, ci, va, x, y0, alpha, beta, slab_cols: int, slab0_cols: int | None = None,
                    beta_last: bool = False, term_slab=None, n_slabs: int | None = None):
    """The multi-slab band layouts' sum, restated on the oracle: each column slab summed in
    the reference's order (oracle.csr_spmv) -- slab 0 from beta*y, later slabs from -0.0 --
    then the slab sums added in slab order in fp32.  beta_last (sm_info.xband_beta_last, the
    band2 / cband hand-off): every slab from -0.0, y = (((beta*y + P_0) + P_1) + ...), beta*y
    as kernel.cc:10-29 forms it (y *= beta unless beta == 1).  Slab 0 covers [0, slab0_cols),
    slab s >= 1 [slab0_cols + (s-1) slab_cols, slab0_cols + s slab_cols)
    (sm_info.xband_slab0_cols / xband_slab_cols; even slabs when slab0_cols is None), unless
    term_slab gives every term's slab.  Bit-exact target for has_xband 2/3/4/5/6 with several slabs."""
    import oracle
    rp = np.asarray(rp, np.int64)
    ci = np.asarray(ci)
    va = np.asarray(va, np.float32)
    y0 = np.asarray(y0, np.float32)
    n = rp.size - 1
    n_cols = x.size
    if term_slab is None:
        s0 = slab_cols if slab0_cols is None else slab0_cols
        n_slabs = 1 + max(0, -(-(n_cols - s0) // slab_cols))
        term_slab = np.where(ci < s0, 0, 1 + (ci.astype(np.int64) - s0) // slab_cols)
    bl = beta_last and n_slabs > 1
    out = (y0 * np.float32(beta) if beta != 1.0 else y0.copy()) if bl else None
    for s in range(n_slabs):
        mask = term_slab == s
        cm = np.concatenate([[0], np.cumsum(mask)])
        rps = np.zeros(n + 1, np.int64)
        rps[1:] = cm[rp[1:]] - cm[rp[:-1]]
        rps = np.cumsum(rps)
        if s == 0 and not bl:
            p = oracle.csr_spmv(rps, ci[mask], va[mask], x, y0, alpha, beta)
        else:
            p = oracle.csr_spmv(rps, ci[mask], va[mask], x, np.full(n, -0.0, np.float32), alpha, 1.0)
        out = p if out is None else (out + p).astype(np.float32)
    return out


def slab_order_for(info, rp, ci, va, x, y0, alpha, beta):
    """slab_order_spmv with the slab geometry and hand-off form the matrix reports."""
    return slab_order_spmv(rp, ci, va, x, y0, alpha, beta, info["xband_slab_cols"], info["xband_slab0_cols"],
                           beta_last=bool(info["xband_beta_last"]))
