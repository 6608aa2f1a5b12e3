"""Sorted sliced-ELL SpMV (sell.cpp + kernels_sell.hip) through the C ABI.

Every row of at most 2048 terms is summed by one lane in stored order, so those rows
are bit-identical to the reference's order (oracle.csr_spmv); longer rows are cut in
2048-term segments whose sums are added in order, checked within 1e-6 * sum|terms|.
"""
import numpy as np
import pytest

import oracle
from gpu_util import (assert_terms_close, bits, skewed_csr, to_dev, to_host, torch_dev,
                      uniform_csr)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sm():
    torch_dev()
    oracle.build()
    import sparsematrix_amd
    sparsematrix_amd.load()
    return sparsematrix_amd


def _sell(sm, rp, ci, va, n_cols, relabel=None, **opts):
    o = dict(layout="no_bands", **opts)
    if relabel is not None:
        o["relabel"] = relabel
    M = sm.SparseMatrix.from_csr(rp, ci, va, n_cols, opts=o)
    info = M.info()
    assert info["sell_slices"] > 0 and info["has_xband"] == 0, info
    return M, info


def _check(M, rp, ci, va, x, y0, alpha, beta, algo="auto", exact_max=None):
    y = to_dev(y0)
    M.spmv(to_dev(x), y, alpha, beta, algo=algo)
    got = to_host(y)
    want = oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta)
    lens = np.diff(np.asarray(rp, np.int64))
    short = lens <= (exact_max if exact_max is not None else lens.max())
    assert np.array_equal(bits(got[short]), bits(want[short])), (alpha, beta)
    _, absum = oracle.csr_spmv_f64(np.asarray(rp, np.int64), ci, va, x, y0, alpha, beta)
    assert_terms_close(got, want, absum)


@pytest.mark.parametrize("n_rows,n_cols,per_row", [(100003, 200001, 16), (5000, 3000, 1),
                                                   (64, 1000, 7), (65, 70, 64), (1, 10, 3)])
def test_sell_uniform_bit_exact(sm, n_rows, n_cols, per_row):
    rp, ci, va = uniform_csr(n_rows, n_cols, per_row, seed=n_rows)
    M, info = _sell(sm, rp, ci, va, n_cols)
    assert info["sell_codebook"] == 1, info   # table values: the 4-byte word form
    rng = np.random.default_rng(1)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y0[::37] = np.nan
    for alpha, beta, algo in ((1.0, 1.0, "auto"), (1.3, 0.7, "sell"), (0.5, 0.0, "auto")):
        _check(M, rp, ci, va, x, y0, alpha, beta, algo)


@pytest.mark.parametrize("relabel", [0, 1])
def test_sell_skewed_rows_and_long_rows(sm, relabel):
    """Power-law row lengths with empty rows and rows past 2048 terms (segmented):
    short rows bit-exact, all rows within the bound; the column relabeling (x
    permuted per SpMV) gives the same bits."""
    rng = np.random.default_rng(7)
    n_rows, n_cols = 60000, 90000
    lengths = np.minimum((rng.pareto(1.2, n_rows) * 3).astype(np.int64), 30000)
    lengths[::7] = 0
    lengths[5] = 9000
    rp, ci, va = skewed_csr(n_rows, n_cols, lengths, seed=8)
    M, info = _sell(sm, rp, ci, va, n_cols, relabel)
    assert info["col_relabel"] == relabel
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    for alpha, beta in ((1.0, 1.0), (1.3, 0.7), (0.5, 0.0)):
        _check(M, rp, ci, va, x, y0, alpha, beta, exact_max=2048)


@pytest.mark.parametrize("skewed", [False, True])
def test_sell_codebook_form(sm, skewed):
    """Values from a <= 255-entry table (the reference's uint8 ids, inf / NaN / -0.0
    among them): the slices hold column | id << 24 words (sell_codebook = 1) and give
    the same bits as the plain column + value form (sell_codebook = 0) and the oracle."""
    rng = np.random.default_rng(21)
    n_rows, n_cols = 40009, 70001
    if skewed:
        lengths = np.minimum((rng.pareto(1.1, n_rows) * 4).astype(np.int64), 7000)
        lengths[::6] = 0
        rp, ci, _ = skewed_csr(n_rows, n_cols, lengths, seed=22)
    else:
        rp, ci, _ = uniform_csr(n_rows, n_cols, 11, seed=23)
    table = rng.uniform(-2, 2, 200).astype(np.float32)
    table[:4] = [np.inf, np.nan, -0.0, 0.0]
    va = table[rng.integers(0, table.size, ci.size)]
    M, info = _sell(sm, rp, ci, va, n_cols, 0)
    assert info["sell_codebook"] == 1, info
    P, pinfo = _sell(sm, rp, ci, va, n_cols, 0, sell_codebook=0)
    assert pinfo["sell_codebook"] == 0 and info["device_bytes"] < pinfo["device_bytes"]
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    x[0] = np.inf                       # what padding words point at
    x[7::5003] = np.nan
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y0[:40] = -0.0
    for alpha, beta in ((1.0, 1.0), (1.7, 0.0), (-0.5, 2.0)):
        ys = []
        for A in (M, P):
            y = to_dev(y0)
            A.spmv(to_dev(x), y, alpha, beta)
            ys.append(to_host(y))
        assert np.array_equal(bits(ys[0]), bits(ys[1])), (alpha, beta)
        lens = np.diff(np.asarray(rp, np.int64))
        want = oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta)
        assert np.array_equal(bits(ys[0][lens <= 2048]), bits(want[lens <= 2048]))


@pytest.mark.parametrize("sigma,streams", [(4096, 8), (4096, 1), (1000, 3)])
def test_sell_sort_windows(sm, sigma, streams):
    """SELL-C-sigma layouts (sell_sigma rows per sort window, sell_streams XCD
    streams of windows): the same per-row order, so the same bits as one window."""
    rng = np.random.default_rng(11)
    n_rows, n_cols = 30011, 40000
    lengths = np.minimum((rng.pareto(1.1, n_rows) * 4).astype(np.int64), 6000)
    lengths[::5] = 0
    rp, ci, va = skewed_csr(n_rows, n_cols, lengths, seed=12)
    M, _ = _sell(sm, rp, ci, va, n_cols, 0, sell_sigma=sigma, sell_streams=streams)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    for alpha, beta in ((1.0, 1.0), (1.3, 0.0)):
        _check(M, rp, ci, va, x, y0, alpha, beta, exact_max=2048)


def test_sell_special_values(sm):
    n_rows, n_cols = 20000, 30000
    rp, ci, va = uniform_csr(n_rows, n_cols, 9, seed=3)
    va = va.copy()
    va[::499] = np.inf
    va[3::701] = np.nan
    va[100:400] = -0.0
    rng = np.random.default_rng(4)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    x[0] = np.inf                       # what every padding slot reads
    x[5::3001] = np.nan
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y0[:50] = -0.0
    M, _ = _sell(sm, rp, ci, va, n_cols)
    for alpha, beta in ((1.0, 1.0), (2.0, 0.0), (0.5, 3.0)):
        y = to_dev(y0)
        M.spmv(to_dev(x), y, alpha, beta)
        assert np.array_equal(bits(to_host(y)), bits(oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta)))


def test_sell_rmat_auto(sm):
    """AUTO without band layouts on an R-MAT graph (scale 20): column relabeling +
    sell; short rows bit-exact, long rows within the bound."""
    torch = torch_dev()
    import sparsematrix_amd.synth as synth
    rp_d, ci_d, va_d = synth.rmat_device(20, 16, seed=4)
    n = 1 << 20
    M = sm.SparseMatrix.from_csr(rp_d, ci_d, va_d, n, opts=dict(layout="no_bands"))
    info = M.info()
    assert info["sell_slices"] > 0 and info["col_relabel"] == 1 and info["sell_codebook"] == 1, info
    rp, ci, va = rp_d.cpu().numpy(), ci_d.cpu().numpy(), va_d.cpu().numpy()
    rng = np.random.default_rng(9)
    x = rng.uniform(-1, 1, n).astype(np.float32)
    y0 = rng.uniform(-1, 1, n).astype(np.float32)
    _check(M, rp, ci, va, x, y0, 1.0, 0.5, exact_max=2048)
