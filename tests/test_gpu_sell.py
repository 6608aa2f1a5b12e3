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
    """R-MAT scale 20 without band layouts: column relabeling + codebook sell, rows of up
    to 2048 terms bit-exact (AUTO builds no hot-column bands); the opt-in split (the
    hottest relabeled columns as codebook bands first, then the sliced ELL) stays
    within 1e-6 * sum|terms| on every row."""
    torch = torch_dev()
    import sparsematrix_amd.synth as synth
    rp_d, ci_d, va_d = synth.rmat_device(20, 16, seed=4)
    n = 1 << 20
    M = sm.SparseMatrix.from_csr(rp_d, ci_d, va_d, n, opts=dict(layout="no_bands"))
    info = M.info()
    assert info["sell_slices"] > 0 and info["col_relabel"] == 1 and info["sell_codebook"] == 1, info
    assert info["hot_cols"] == 0, info
    rp, ci, va = rp_d.cpu().numpy(), ci_d.cpu().numpy(), va_d.cpu().numpy()
    rng = np.random.default_rng(9)
    x = rng.uniform(-1, 1, n).astype(np.float32)
    y0 = rng.uniform(-1, 1, n).astype(np.float32)
    _check(M, rp, ci, va, x, y0, 1.0, 0.5, exact_max=2048)
    H = sm.SparseMatrix.from_csr(rp_d, ci_d, va_d, n, opts=dict(layout="no_bands", hot_cols=32768))
    hinfo = H.info()
    assert hinfo["hot_cols"] == 32768 and hinfo["col_relabel"] == 1, hinfo
    for alpha, beta in ((1.0, 0.5), (1.3, 0.0), (-0.7, 1.0)):
        _check(H, rp, ci, va, x, y0, alpha, beta, exact_max=0)
        _check(H, rp, ci, va, x, y0, alpha, beta, algo="sell", exact_max=0)


@pytest.mark.parametrize("hot", [8192, 40000])
def test_hot_bands_forced_skewed(sm, hot):
    """Forced hot-column split on a power-law-column matrix (relabeled): hot terms through
    the codebook bands (one or several windows), the rest through the sliced ELL with its
    long-row segments; special values and beta = 0 with NaN in y."""
    rng = np.random.default_rng(hot)
    n_rows, n_cols, per = 300000, 1 << 20, 12
    label = rng.permutation(n_cols).astype(np.int32)
    raw = np.minimum(rng.zipf(1.2, (n_rows, per)) - 1, n_cols - 1)
    cols = np.sort(label[raw], axis=1)
    keep = np.ones_like(cols, bool)
    keep[:, 1:] = cols[:, 1:] != cols[:, :-1]
    keep[7] = False                      # an empty row
    lens = keep.sum(axis=1)
    ci = cols[keep].astype(np.int32)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    table = rng.uniform(-1, 1, 255).astype(np.float32)
    table[:3] = [np.inf, -0.0, 0.0]
    va = table[rng.integers(0, 255, ci.size)]
    M = sm.SparseMatrix.from_csr(rp, ci, va, n_cols, opts=dict(layout="no_bands", relabel=1, hot_cols=hot))
    info = M.info()
    assert info["hot_cols"] == hot and info["sell_slices"] > 0, info
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y0[::101] = np.nan
    for alpha, beta in ((1.0, 1.0), (0.5, 0.0), (2.0, 3.0)):
        _check(M, rp, ci, va, x, y0, alpha, beta, exact_max=0)


def test_config4_rmat24_auto_vs_oracle(sm):
    """BASELINE config 4 at full size, exactly as bench.py builds it: Graph500 R-MAT
    scale 24, edgefactor 16, seed 4 (263 M terms, rows up to 238 465 terms), AUTO =
    column relabeling + codebook sliced ELL with 2048-term segments.  Every row of up to
    2048 terms is bit-identical to the reference order (oracle), the longer rows (their
    segment sums added in order) and the opt-in hot-column split within 1e-6 * sum|terms|."""
    torch = torch_dev()
    import sparsematrix_amd.synth as synth
    rp_d, ci_d, va_d = synth.rmat_device(24, 16, seed=4)
    n = 1 << 24
    M = sm.SparseMatrix.from_csr(rp_d, ci_d, va_d, n)
    info = M.info()
    assert info["sell_slices"] > 0 and info["col_relabel"] == 1 and info["sell_codebook"] == 1, info
    assert info["max_row_nnz"] > 2048 and info["hot_cols"] == 0, info
    E = sm.SparseMatrix.from_csr(rp_d, ci_d, va_d, n, opts=dict(hot_cols=32768))
    assert E.info()["hot_cols"] == 32768
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y0 = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y, ye = y0.clone(), y0.clone()
    M.spmv(x, y, 1.0, 0.5)
    E.spmv(x, ye, 1.0, 0.5)
    got, got_e = to_host(y), to_host(ye)
    del M, E
    rp, ci, va = rp_d.cpu().numpy(), ci_d.cpu().numpy(), va_d.cpu().numpy()
    del rp_d, ci_d, va_d
    xh, y0h = to_host(x), to_host(y0)
    want = oracle.csr_spmv_mt(rp, ci, va, xh, y0h, 1.0, 0.5, threads=16)
    lens = np.diff(rp.astype(np.int64))
    short = lens <= 2048
    # AUTO: every row of <= 2048 terms in the reference's order
    assert np.array_equal(bits(got[short]), bits(want[short]))
    # the opt-in hot bands, and the long rows: the Sum|terms| bound
    _, absum = oracle.csr_spmv_f64(rp.astype(np.int64), ci, va, xh, y0h, 1.0, 0.5)
    assert_terms_close(got, want, absum)
    assert_terms_close(got_e, want, absum)
