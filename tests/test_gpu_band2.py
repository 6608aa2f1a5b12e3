"""Balanced-band SpMV (has_xband == 4: band2.cpp + kernels_band2.hip) through the C ABI.

Bit-exact targets: with one slab, the reference's order (oracle.csr_spmv); with
several, the slab-order restatement (gpu_util.slab_order_spmv: every slab in the
reference's order, slab sums added in slab order) -- so every case is compared
bit for bit, and also checked against the reference within 1e-6 * sum|terms|.
"""
import numpy as np
import pytest

import oracle
from gpu_util import (assert_terms_close, bits, slab_order_spmv, to_dev, to_host, torch_dev,
                      uniform_csr, with_env)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sm():
    torch_dev()
    oracle.build()
    import sparsematrix_amd
    sparsematrix_amd.load()
    return sparsematrix_amd


def _band2(sm, rp, ci, va, n_cols, slabs=None):
    def make():
        return with_env("SM_XBAND_KIND", "band2", lambda: with_env(
            "SM_XBAND", "1", lambda: sm.SparseMatrix.from_csr(rp, ci, va, n_cols)))
    M = with_env("SM_BAND2_SLABS", str(slabs), make) if slabs else make()
    info = M.info()
    assert info["has_xband"] == 4, info
    return M, info


def _check(M, info, rp, ci, va, x, y0, alpha, beta, algo="xband"):
    y = to_dev(y0)
    M.spmv(to_dev(x), y, alpha, beta, algo=algo)
    got = to_host(y)
    if info["xband_slabs"] == 1:
        want = oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta)
    else:
        want = slab_order_spmv(rp, ci, va, x, y0, alpha, beta, info["xband_slab_cols"])
    assert np.array_equal(bits(got), bits(want)), (alpha, beta, info["xband_slabs"])
    ref = oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta)
    _, absum = oracle.csr_spmv_f64(rp, ci, va, x, y0, alpha, beta)
    assert_terms_close(got, ref, absum)


SHAPES = [(200003, 300001, 16), (9000, 70001, 40), (5000, 1000, 5), (40000, 20000, 3),
          (70000, 1000003, 16), (1, 50000, 30), (16384, 8192, 1)]


@pytest.mark.parametrize("n_rows,n_cols,per_row", SHAPES)
@pytest.mark.parametrize("slabs", [1, None])
def test_band2_vs_oracle(sm, n_rows, n_cols, per_row, slabs):
    rp, ci, va = uniform_csr(n_rows, n_cols, per_row, seed=n_rows + n_cols)
    M, info = _band2(sm, rp, ci, va, n_cols, slabs)
    if slabs == 1:
        assert info["xband_slabs"] == 1
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y0[::97] = np.nan
    for alpha, beta, algo in ((1.0, 1.0, "xband"), (1.3, 0.7, "auto"), (0.5, 0.0, "xband")):
        _check(M, info, rp, ci, va, x, y0, alpha, beta, algo)


def test_band2_long_segments_cut(sm):
    """Rows with 40 consecutive columns: a band holds at most 14 terms of one row, so
    the builder cuts bands inside such runs; order and results stay exact."""
    n_rows, n_cols, w = 6000, 7000, 40
    starts = np.random.default_rng(3).integers(0, n_cols - w, n_rows)
    ci = (starts[:, None] + np.arange(w)[None, :]).reshape(-1).astype(np.int32)
    rp = np.arange(0, n_rows * w + 1, w, dtype=np.int32)
    va = np.random.default_rng(4).uniform(-1, 1, ci.size).astype(np.float32)
    for slabs in (1, None):
        M, info = _band2(sm, rp, ci, va, n_cols, slabs)
        x = np.random.default_rng(6).uniform(-1, 1, n_cols).astype(np.float32)
        y0 = np.random.default_rng(7).uniform(-1, 1, n_rows).astype(np.float32)
        _check(M, info, rp, ci, va, x, y0, 1.0, 0.5)


def test_band2_ragged_rows_and_empty_regions(sm):
    """Empty rows, one dense row, column ranges without terms (bands skip them)."""
    rng = np.random.default_rng(11)
    n_rows, n_cols = 40000, 600000
    lens = rng.integers(0, 12, n_rows)
    lens[::50] = 0
    lens[777] = 3000
    rows = []
    for r in range(n_rows):
        lo, hi = (0, 100000) if r % 2 else (400000, 600000)
        k = min(int(lens[r]), hi - lo)
        rows.append(np.sort(rng.choice(np.arange(lo, hi), k, replace=False)))
    rp = np.zeros(n_rows + 1, np.int32)
    rp[1:] = np.cumsum([len(c) for c in rows])
    ci = np.concatenate(rows).astype(np.int32)
    va = rng.uniform(-1, 1, ci.size).astype(np.float32)
    for slabs in (1, None):
        M, info = _band2(sm, rp, ci, va, n_cols, slabs)
        x = rng.uniform(-1, 1, n_cols).astype(np.float32)
        y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
        _check(M, info, rp, ci, va, x, y0, 1.3, 0.7)


def test_band2_special_values_and_signed_zeros(sm):
    n_rows, n_cols = 30000, 50000
    rp, ci, va = uniform_csr(n_rows, n_cols, 6, seed=77)
    va = va.copy()
    va[::997] = np.inf
    va[5::1009] = np.nan
    va[6 * 100:6 * 200] = -0.0
    rng = np.random.default_rng(8)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    x[0] = np.inf                      # what every dummy lane reads
    x[1::4999] = -np.inf
    x[2::7001] = np.nan
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y0[:300] = -0.0
    for slabs in (1, None):
        M, info = _band2(sm, rp, ci, va, n_cols, slabs)
        for alpha, beta in ((1.0, 1.0), (0.5, 0.0), (2.0, 3.0)):
            y = to_dev(y0)
            M.spmv(to_dev(x), y, alpha, beta, algo="xband")
            got = to_host(y)
            want = (oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta) if info["xband_slabs"] == 1
                    else slab_order_spmv(rp, ci, va, x, y0, alpha, beta, info["xband_slab_cols"]))
            assert np.array_equal(bits(got), bits(want))


def test_band2_repeated_launches_reset_handoff(sm):
    """Back-to-back SpMVs on one stream: the slab hand-off's control words return to
    zero after every launch, so repeated products are bit-identical."""
    torch = torch_dev()
    n_rows, n_cols = 300000, 400000
    rp, ci, va = uniform_csr(n_rows, n_cols, 16, seed=21)
    M, info = _band2(sm, rp, ci, va, n_cols)
    assert info["xband_slabs"] > 1
    rng = np.random.default_rng(22)
    x = to_dev(rng.uniform(-1, 1, n_cols).astype(np.float32))
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    ys = [to_dev(y0) for _ in range(6)]
    for y in ys:
        M.spmv(x, y, 1.0, 0.5)
    torch.cuda.synchronize()
    first = bits(to_host(ys[0]))
    for y in ys[1:]:
        assert np.array_equal(bits(to_host(y)), first)
    want = slab_order_spmv(rp, ci, va, to_host(x), y0, 1.0, 0.5, info["xband_slab_cols"])
    assert np.array_equal(first, bits(want))


def test_band2_config2_equals_blocked(sm):
    """BASELINE config 2 (2^20 x 2^20, 16 terms/row): band2 and the blocked kind use
    the same 4 slabs of 262144 columns and sum each in the reference's order, so
    their results are bit-identical; sampled rows match the slab-order oracle."""
    torch = torch_dev()
    import sparsematrix_amd.synth as synth
    n = 1 << 20
    rp, ci, va = synth.uniform_rows_device(n, n, 16, seed=2)
    Mb2 = with_env("SM_XBAND_KIND", "band2", lambda: sm.SparseMatrix.from_csr(rp, ci, va, n))
    Mbl = with_env("SM_XBAND_KIND", "blocked", lambda: sm.SparseMatrix.from_csr(rp, ci, va, n))
    i2, ib = Mb2.info(), Mbl.info()
    assert i2["has_xband"] == 4 and ib["has_xband"] == 2
    assert i2["xband_slabs"] == ib["xband_slabs"] == 4
    assert i2["xband_slab_cols"] == ib["xband_slab_cols"] == 262144
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y0 = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y2, yb = y0.clone(), y0.clone()
    Mb2.spmv(x, y2, 1.0, 0.5)
    Mbl.spmv(x, yb, 1.0, 0.5)
    torch.cuda.synchronize()
    assert torch.equal(y2.view(torch.int32), yb.view(torch.int32))
