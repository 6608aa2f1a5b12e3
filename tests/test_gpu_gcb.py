"""Gathered chunk bands (has_xband == 6, gcb.cpp + kernels_gcb.hip) through the C ABI:
the layout for wide matrices (BASELINE config 5's rank slices), forced here with
layout="gcb" on small and irregular shapes.

Bit-exact targets: with one slab the reference's order (oracle.csr_spmv: every row's
terms in ascending column order, kernel.cc:780-796); with several, the slab-order
restatement (gpu_util.slab_order_spmv) -- and always within 1e-6 * sum|terms| of the
reference."""
import numpy as np
import pytest

import oracle
from gpu_util import assert_terms_close, bits, slab_order_spmv, to_dev, to_host, torch_dev, uniform_csr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sm():
    torch_dev()
    oracle.build()
    import sparsematrix_amd
    sparsematrix_amd.load()
    return sparsematrix_amd


def _gcb(sm, rp, ci, va, n_cols, slabs=0):
    M = sm.SparseMatrix.from_csr(rp, ci, va, n_cols, opts=dict(layout="gcb", band_slabs=slabs))
    info = M.info()
    assert info["has_xband"] == 6, info
    return M, info


def _check(M, info, rp, ci, va, x, y0, alpha, beta, algo="xband"):
    y = to_dev(y0)
    M.spmv(to_dev(x), y, alpha, beta, algo=algo)
    got = to_host(y)
    if info["xband_slabs"] == 1:
        want = oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta)
    else:
        want = slab_order_spmv(rp, ci, va, x, y0, alpha, beta, info["xband_slab_cols"], info["xband_slab0_cols"])
    assert np.array_equal(bits(got), bits(want)), (alpha, beta, info["xband_slabs"])
    ref = oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta)
    _, absum = oracle.csr_spmv_f64(rp, ci, va, x, y0, alpha, beta)
    assert_terms_close(got, ref, absum)


SHAPES = [(200003, 3000001, 16), (70000, 1000003, 16), (9000, 70001, 40), (5000, 1000, 5),
          (1, 50000, 30), (40000, 20000, 3), (300000, 8000000, 4)]


@pytest.mark.parametrize("n_rows,n_cols,per_row", SHAPES)
@pytest.mark.parametrize("slabs", [1, 0, 3])
def test_gcb_vs_oracle(sm, n_rows, n_cols, per_row, slabs):
    rp, ci, va = uniform_csr(n_rows, n_cols, per_row, seed=n_rows + n_cols)
    M, info = _gcb(sm, rp, ci, va, n_cols, slabs)
    if slabs == 1:
        assert info["xband_slabs"] == 1
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y0[::97] = np.nan
    for alpha, beta, algo in ((1.0, 1.0, "xband"), (1.3, 0.7, "auto"), (0.5, 0.0, "xband")):
        _check(M, info, rp, ci, va, x, y0, alpha, beta, algo)


def test_gcb_long_segments_and_hub_columns(sm):
    """Rows of 90 consecutive columns (a band holds at most 63 terms of one row, so the
    builder cuts inside the run), and hub columns shared by every row (more than a band's
    2016 terms in one column: the column's rows are split over several bands)."""
    rng = np.random.default_rng(3)
    n_rows, n_cols, w = 6000, 700000, 90
    rows = []
    for r in range(n_rows):
        s = int(rng.integers(0, n_cols - w - 10))
        cols = np.arange(s, s + w)
        cols = np.union1d(cols, [5, 600000])          # two hub columns in every row
        rows.append(cols)
    rp = np.zeros(n_rows + 1, np.int32)
    rp[1:] = np.cumsum([len(c) for c in rows])
    ci = np.concatenate(rows).astype(np.int32)
    va = rng.uniform(-1, 1, ci.size).astype(np.float32)
    for slabs in (1, 0):
        M, info = _gcb(sm, rp, ci, va, n_cols, slabs)
        x = rng.uniform(-1, 1, n_cols).astype(np.float32)
        y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
        _check(M, info, rp, ci, va, x, y0, 1.0, 0.5)


def test_gcb_ragged_special_values(sm):
    """Empty rows, a dense row, empty column ranges, inf / NaN / -0.0 in x, values and y."""
    rng = np.random.default_rng(11)
    n_rows, n_cols = 40000, 2000000
    lens = rng.integers(0, 12, n_rows)
    lens[::50] = 0
    lens[777] = 3000
    rows = []
    for r in range(n_rows):
        lo, hi = (0, 300000) if r % 2 else (1200000, 2000000)
        rows.append(np.sort(rng.choice(np.arange(lo, hi), int(lens[r]), replace=False)))
    rp = np.zeros(n_rows + 1, np.int32)
    rp[1:] = np.cumsum([len(c) for c in rows])
    ci = np.concatenate(rows).astype(np.int32)
    va = rng.uniform(-1, 1, ci.size).astype(np.float32)
    va[::101] = -0.0
    va[7::1009] = np.inf
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    x[::1013] = -0.0
    x[3::100003] = np.nan
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y0[::89] = -0.0
    for slabs in (1, 0):
        M, info = _gcb(sm, rp, ci, va, n_cols, slabs)
        y = to_dev(y0)
        M.spmv(to_dev(x), y, 1.3, 0.0)
        got = to_host(y)
        want = (oracle.csr_spmv(rp, ci, va, x, y0, 1.3, 0.0) if info["xband_slabs"] == 1
                else slab_order_spmv(rp, ci, va, x, y0, 1.3, 0.0, info["xband_slab_cols"], info["xband_slab0_cols"]))
        assert np.array_equal(bits(got), bits(want)), info["xband_slabs"]


def test_gcb_repeated_launches_reset_handoff(sm):
    rp, ci, va = uniform_csr(100000, 4000000, 16, seed=9)
    M, info = _gcb(sm, rp, ci, va, 4000000, 4)
    assert info["xband_slabs"] == 4
    torch = torch_dev()
    x = torch.rand(4000000, device="cuda") * 2 - 1
    y0 = np.random.default_rng(2).uniform(-1, 1, 100000).astype(np.float32)
    ys = [to_dev(y0) for _ in range(6)]
    for y in ys:
        M.spmv(x, y, 1.0, 0.5)
    want = slab_order_spmv(rp, ci, va, to_host(x), y0, 1.0, 0.5, info["xband_slab_cols"], info["xband_slab0_cols"])
    for y in ys:
        assert np.array_equal(bits(to_host(y)), bits(want))
