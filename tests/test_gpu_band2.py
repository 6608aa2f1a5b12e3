"""Balanced-band SpMV through the C ABI: band2 (has_xband == 4, 8-byte entries) and
cband (has_xband == 5, 4-byte codebook words), band2.cpp + kernels_band2.hip.

Bit-exact targets: with one slab, the reference's order (oracle.csr_spmv); with
several, the slab-order restatement (gpu_util.slab_order_spmv: every slab in the
reference's order, slab sums added in slab order) -- so every case is compared
bit for bit, and also checked against the reference within 1e-6 * sum|terms|.
"""
import numpy as np
import pytest

import oracle
from gpu_util import (assert_terms_close, bits, slab_order_for, to_dev, to_host, torch_dev,
                      uniform_csr)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sm():
    torch_dev()
    oracle.build()
    import sparsematrix_amd
    sparsematrix_amd.load()
    return sparsematrix_amd


KINDS = {"band2": 4, "cband": 5}


def _codebook(va, n=200, seed=0):
    """The values requantised onto an n-entry table (cband needs <= 255 distinct)."""
    table = np.random.default_rng(seed).uniform(-1, 1, n).astype(np.float32)
    ids = np.random.default_rng(seed + 1).integers(0, n, va.size)
    return table[ids].astype(np.float32)


def _band2(sm, rp, ci, va, n_cols, slabs=None, kind="band2", tall=0):
    M = sm.SparseMatrix.from_csr(rp, ci, va, n_cols,
                                 opts=dict(layout=kind, band_tall=tall, band_slabs=slabs or 0))
    info = M.info()
    assert info["has_xband"] == KINDS[kind], info
    assert info["xband_block_rows"] <= 16384, info
    return M, info


def _check(M, info, rp, ci, va, x, y0, alpha, beta, algo="xband"):
    y = to_dev(y0)
    M.spmv(to_dev(x), y, alpha, beta, algo=algo)
    got = to_host(y)
    if info["xband_slabs"] == 1:
        want = oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta)
    else:
        want = slab_order_for(info, rp, ci, va, x, y0, alpha, beta)
    assert np.array_equal(bits(got), bits(want)), (alpha, beta, info["xband_slabs"])
    ref = oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta)
    _, absum = oracle.csr_spmv_f64(rp, ci, va, x, y0, alpha, beta)
    assert_terms_close(got, ref, absum)


SHAPES = [(200003, 300001, 16), (9000, 70001, 40), (5000, 1000, 5), (40000, 20000, 3),
          (70000, 1000003, 16), (1, 50000, 30), (16384, 8192, 1)]


@pytest.mark.parametrize("n_rows,n_cols,per_row", SHAPES)
@pytest.mark.parametrize("slabs", [1, None])
@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("tall", [0, 6])
def test_band2_vs_oracle(sm, n_rows, n_cols, per_row, slabs, kind, tall):
    """tall: 0 the default (dma3: a loader wave stages x; both encodings), 6 wide (the fallback
    when dma3's bands would be mostly padding)."""
    rp, ci, va = uniform_csr(n_rows, n_cols, per_row, seed=n_rows + n_cols)
    M, info = _band2(sm, rp, ci, va, n_cols, slabs, kind, tall)
    if slabs == 1:
        assert info["xband_slabs"] == 1
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y0[::97] = np.nan
    for alpha, beta, algo in ((1.0, 1.0, "xband"), (1.3, 0.7, "auto"), (0.5, 0.0, "xband")):
        _check(M, info, rp, ci, va, x, y0, alpha, beta, algo)


@pytest.mark.parametrize("kind,w", [("band2", 40), ("cband", 40), ("cband", 90)])
def test_band2_long_segments_cut(sm, kind, w):
    """Rows of w consecutive columns: a band holds at most 14 (band2) / 63 (cband)
    terms of one row, so the builder cuts bands inside longer runs; cband's 40-term
    segments stay whole and run 39 rounds of the lane-to-lane sum."""
    n_rows, n_cols = 6000, 7000
    starts = np.random.default_rng(3).integers(0, n_cols - w, n_rows)
    ci = (starts[:, None] + np.arange(w)[None, :]).reshape(-1).astype(np.int32)
    rp = np.arange(0, n_rows * w + 1, w, dtype=np.int32)
    va = np.random.default_rng(4).uniform(-1, 1, ci.size).astype(np.float32)
    if kind == "cband":
        va = _codebook(va)
    for slabs in (1, None):
        M, info = _band2(sm, rp, ci, va, n_cols, slabs, kind)
        x = np.random.default_rng(6).uniform(-1, 1, n_cols).astype(np.float32)
        y0 = np.random.default_rng(7).uniform(-1, 1, n_rows).astype(np.float32)
        _check(M, info, rp, ci, va, x, y0, 1.0, 0.5)


@pytest.mark.parametrize("kind", list(KINDS))
def test_band2_ragged_rows_and_empty_regions(sm, kind):
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
    if kind == "cband":
        va = _codebook(va)
    for slabs in (1, None):
        M, info = _band2(sm, rp, ci, va, n_cols, slabs, kind)
        x = rng.uniform(-1, 1, n_cols).astype(np.float32)
        y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
        _check(M, info, rp, ci, va, x, y0, 1.3, 0.7)


@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("tall", [0, 6])
def test_band2_special_values_and_signed_zeros(sm, kind, tall):
    n_rows, n_cols = 30000, 50000
    rp, ci, va = uniform_csr(n_rows, n_cols, 6, seed=77,
                             table=np.random.default_rng(1).uniform(-1, 1, 250).astype(np.float32))
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
        M, info = _band2(sm, rp, ci, va, n_cols, slabs, kind, tall)
        for alpha, beta in ((1.0, 1.0), (0.5, 0.0), (2.0, 3.0)):
            y = to_dev(y0)
            M.spmv(to_dev(x), y, alpha, beta, algo="xband")
            got = to_host(y)
            want = (oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta) if info["xband_slabs"] == 1
                    else slab_order_for(info, rp, ci, va, x, y0, alpha, beta))
            assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("tall", [0, 6])
def test_band2_repeated_launches_reset_handoff(sm, kind, tall):
    """Back-to-back SpMVs on one stream: the slab hand-off's control words return to
    zero after every launch, so repeated products are bit-identical."""
    torch = torch_dev()
    n_rows, n_cols = 300000, 400000
    rp, ci, va = uniform_csr(n_rows, n_cols, 16, seed=21)
    M, info = _band2(sm, rp, ci, va, n_cols, kind=kind, tall=tall)
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
    want = slab_order_for(info, rp, ci, va, to_host(x), y0, 1.0, 0.5)
    assert np.array_equal(first, bits(want))


@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("permille", [900, 960])
def test_band2_narrow_slab0_vs_oracle(sm, kind, permille):
    """sm_build_opts.band_slab0_permille: slab 0 narrower than the even share, the other
    slabs split the rest; bit-identical to the slab-order restatement on the reported
    boundaries (sm_info.xband_slab0_cols / xband_slab_cols)."""
    n_rows, n_cols = 200003, 300001
    rp, ci, va = uniform_csr(n_rows, n_cols, 16, seed=41)
    M = sm.SparseMatrix.from_csr(rp, ci, va, n_cols, opts=dict(layout=kind, band_slab0_permille=permille))
    info = M.info()
    assert info["has_xband"] == KINDS[kind] and info["xband_slabs"] > 1, info
    assert info["xband_slab0_cols"] < info["xband_slab_cols"], info
    assert info["xband_slab0_cols"] + (info["xband_slabs"] - 1) * info["xband_slab_cols"] >= n_cols, info
    rng = np.random.default_rng(42)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    _check(M, info, rp, ci, va, x, y0, 1.3, 0.7)


@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("slabs", [3, 5])
def test_handoff_counter_across_32bit_boundary(sm, kind, slabs):
    """the epoch hand-off's launch counter.  A launch's generation is
    g = started / S; with a 32-bit counter and S not dividing 2^32 the launch that crossed
    the wrap gave its tiles different g and hung.  The counter is 64-bit now: seeded just
    below 2^32 (a whole number of launches), four launches cross the boundary and every
    product stays bit-identical to the slab-order oracle."""
    import ctypes
    torch = torch_dev()
    n_rows, n_cols = 100000, 400000
    rp, ci, va = uniform_csr(n_rows, n_cols, 16, seed=31)
    M, info = _band2(sm, rp, ci, va, n_cols, slabs, kind)
    assert info["xband_slabs"] == slabs, info
    seed = ((1 << 32) - 1) // slabs * slabs - slabs   # two launches below the 32-bit boundary
    L = sm._lib.load()
    assert L.sm_debug_seed_handoff(M._require(), ctypes.c_uint64(seed)) == 0
    assert L.sm_debug_seed_handoff(M._require(), ctypes.c_uint64(seed + 1)) != 0
    rng = np.random.default_rng(32)
    x = to_dev(rng.uniform(-1, 1, n_cols).astype(np.float32))
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    want = bits(slab_order_for(info, rp, ci, va, to_host(x), y0, 1.0, 0.5))
    ys = [to_dev(y0) for _ in range(4)]
    for y in ys:
        M.spmv(x, y, 1.0, 0.5)
    torch.cuda.synchronize()
    for y in ys:
        assert np.array_equal(bits(to_host(y)), want)


@pytest.mark.parametrize("n_rows,n_cols,per_row", SHAPES)
def test_cband_dma3_vs_oracle(sm, n_rows, n_cols, per_row):
    """The dma3 geometry (a loader wave stages 7680-column x windows by LDS-DMA into three
    buffers, 15 waves apply 30-chunk bands): bit-identical to the slab-order oracle."""
    rp, ci, va = uniform_csr(n_rows, n_cols, per_row, seed=n_rows + 5 * n_cols)
    for slabs in (1, None):
        M, info = _band2(sm, rp, ci, va, n_cols, slabs, "cband", 4)
        assert info["xband_block_rows"] <= 16384, info
        rng = np.random.default_rng(9)
        x = rng.uniform(-1, 1, n_cols).astype(np.float32)
        y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
        y0[::89] = np.nan
        for alpha, beta in ((1.0, 0.5), (1.3, 0.0), (1.0, 1.0)):
            _check(M, info, rp, ci, va, x, y0, alpha, beta)


def test_cband_dma3_special_values_and_repeats(sm):
    """dma3 with inf / NaN / -0.0 in values, x and y, unaligned windows past n_cols, and six
    back-to-back launches (the hand-off's epoch words) all equal to the oracle."""
    torch = torch_dev()
    n_rows, n_cols = 300000, 400003
    rp, ci, va = uniform_csr(n_rows, n_cols, 16, seed=31,
                             table=np.random.default_rng(2).uniform(-1, 1, 250).astype(np.float32))
    va = va.copy()
    va[::997] = np.inf
    va[5::1009] = -0.0
    M, info = _band2(sm, rp, ci, va, n_cols, None, "cband", 4)
    assert info["xband_slabs"] > 1, info
    rng = np.random.default_rng(32)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    x[1::4999] = -np.inf
    x[2::7001] = np.nan
    x[-1] = np.inf                     # the last column, inside the last window
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y0[:300] = -0.0
    want = slab_order_for(info, rp, ci, va, x, y0, 1.0, 0.5)
    xd = to_dev(x)
    ys = [to_dev(y0) for _ in range(6)]
    for y in ys:
        M.spmv(xd, y, 1.0, 0.5)
    torch.cuda.synchronize()
    for y in ys:
        assert np.array_equal(bits(to_host(y)), bits(want))


@pytest.mark.parametrize("tall", [4, 6])
def test_cband_dma3_config2_vs_slab_oracle(sm, tall):
    """Config 2 in the dma3 geometry (tall 4) and in the wide one (tall 6): bit-identical to
    the 4-slab restatement."""
    torch = torch_dev()
    import sparsematrix_amd.synth as synth
    n = 1 << 20
    rp, ci, va = synth.uniform_rows_device(n, n, 16, seed=2)
    M = sm.SparseMatrix.from_csr(rp, ci, va, n, opts=dict(layout="cband", band_tall=tall))
    info = M.info()
    assert info["has_xband"] == 5 and info["xband_block_rows"] == 16384, info
    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y0 = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y = y0.clone()
    M.spmv(x, y, 1.0, 0.5)
    want = slab_order_for(info, rp.cpu().numpy(), ci.cpu().numpy(), va.cpu().numpy(), to_host(x), to_host(y0),
                          1.0, 0.5)
    assert np.array_equal(bits(to_host(y)), bits(want))


def test_band2_config2_equals_blocked(sm):
    """BASELINE config 2 (2^20 x 2^20, 16 terms/row): cband, band2 and the blocked kind
    built on the same 4 even slabs of 262144 columns sum each in the reference's order, so
    cband and band2 are bit-identical; the blocked kind too unless band2 / cband add beta*y
    in the combine (sm_info.xband_beta_last), then both are within the bound."""
    torch = torch_dev()
    import sparsematrix_amd.synth as synth
    n = 1 << 20
    rp, ci, va = synth.uniform_rows_device(n, n, 16, seed=2)
    Mcb = sm.SparseMatrix.from_csr(rp, ci, va, n)
    Mb2 = sm.SparseMatrix.from_csr(rp, ci, va, n, opts=dict(layout="band2"))
    Mbl = sm.SparseMatrix.from_csr(rp, ci, va, n, opts=dict(layout="blocked"))
    ic, i2, ib = Mcb.info(), Mb2.info(), Mbl.info()
    assert ic["has_xband"] == 5 and i2["has_xband"] == 4 and ib["has_xband"] == 2
    assert ic["xband_slabs"] == i2["xband_slabs"] == ib["xband_slabs"] == 4
    assert ic["xband_slab_cols"] == i2["xband_slab_cols"] == ib["xband_slab_cols"] == 262144
    assert ic["xband_slab0_cols"] == i2["xband_slab0_cols"] == ib["xband_slab0_cols"] == 262144
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y0 = torch.rand(n, device="cuda", generator=g) * 2 - 1
    yc, y2, yb = y0.clone(), y0.clone(), y0.clone()
    Mcb.spmv(x, yc, 1.3, 0.5)
    Mb2.spmv(x, y2, 1.3, 0.5)
    Mbl.spmv(x, yb, 1.3, 0.5)
    torch.cuda.synchronize()
    assert torch.equal(yc.view(torch.int32), y2.view(torch.int32))
    if not ic["xband_beta_last"]:
        assert torch.equal(yc.view(torch.int32), yb.view(torch.int32))
    else:
        # The blocked kind starts slab 0 from beta*y, band2 / cband add beta*y first in the
        # combine: the same four slab sums in another order, both within the bound.
        assert i2["xband_beta_last"] and not ib["xband_beta_last"]
        rph, cih, vah = rp.cpu().numpy(), ci.cpu().numpy(), va.cpu().numpy()
        xh, y0h = to_host(x), to_host(y0)
        ref = oracle.csr_spmv_mt(rph, cih, vah, xh, y0h, 1.3, 0.5, threads=16)
        _, absum = oracle.csr_spmv_f64(rph, cih, vah, xh, y0h, 1.3, 0.5)
        assert_terms_close(to_host(yc), ref, absum)
        assert_terms_close(to_host(yb), ref, absum)


def test_cband_falls_back_without_codebook(sm):
    """More than 255 distinct values: AUTO builds band2 (8-byte entries) instead."""
    rp, ci, va = uniform_csr(50000, 60000, 8, seed=5)
    va = np.random.default_rng(6).uniform(-1, 1, va.size).astype(np.float32)
    M = sm.SparseMatrix.from_csr(rp, ci, va, 60000, opts=dict(layout="bands"))
    assert M.info()["has_xband"] == 4


def test_config2_auto_full_size_vs_oracle(sm):
    """BASELINE config 2 exactly as bench.py runs it (2^20 x 2^20, 16 distinct columns
    per row, seed 2; AUTO = cband, 4 slabs of 262144 columns, alpha 1, beta 0.5):
    bit-identical to the 4-slab restatement of the reference order on the oracle, and
    within 1e-6 * sum|terms| of the reference's own per-row order (oracle.csr_spmv)."""
    torch = torch_dev()
    import sparsematrix_amd.synth as synth
    n = 1 << 20
    rp, ci, va = synth.uniform_rows_device(n, n, 16, seed=2)
    M = sm.SparseMatrix.from_csr(rp, ci, va, n)
    info = M.info()
    assert info["has_xband"] == 5 and info["xband_slabs"] == 4, info
    assert info["xband_slab0_cols"] == info["xband_slab_cols"] == 262144, info
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y0 = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y = y0.clone()
    M.spmv(x, y, 1.0, 0.5)
    got = to_host(y)
    rph, cih, vah = rp.cpu().numpy(), ci.cpu().numpy(), va.cpu().numpy()
    xh, y0h = to_host(x), to_host(y0)
    want = slab_order_for(info, rph, cih, vah, xh, y0h, 1.0, 0.5)
    assert np.array_equal(bits(got), bits(want))
    ref = oracle.csr_spmv_mt(rph, cih, vah, xh, y0h, 1.0, 0.5, threads=16)
    _, absum = oracle.csr_spmv_f64(rph, cih, vah, xh, y0h, 1.0, 0.5)
    assert_terms_close(got, ref, absum)
    # normwise too (<= 1e-6 relative in the 2-norm)
    assert np.linalg.norm(got.astype(np.float64) - ref) <= 1e-6 * np.linalg.norm(ref)


@pytest.mark.parametrize("kind", list(KINDS))
def test_band2_dense_columns_split_by_rows(sm, kind):
    """Hub columns: every row holds column 4097 and every third row column 9000, so
    one column of one 16K-row block needs more than a band's 32 chunks.  The builder
    splits such a column by rows over one-column bands (it used to loop forever);
    AUTO and the forced kinds stay bit-exact against the (slab-order) oracle."""
    n_rows, n_cols = 40000, 20000
    rng = np.random.default_rng(12)
    rows = []
    for r in range(n_rows):
        c = {4097, *rng.integers(0, n_cols, 6).tolist()}
        if r % 3 == 0:
            c.add(9000)
        rows.append(np.array(sorted(c), np.int32))
    rp = np.zeros(n_rows + 1, np.int32)
    rp[1:] = np.cumsum([len(c) for c in rows])
    ci = np.concatenate(rows)
    va = _codebook(rng.uniform(-1, 1, ci.size).astype(np.float32))
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    for slabs in (1, None):
        M, info = _band2(sm, rp, ci, va, n_cols, slabs, kind)
        _check(M, info, rp, ci, va, x, y0, 1.3, 0.7)
    A = sm.SparseMatrix.from_csr(rp, ci, va, n_cols)        # AUTO builds (and serves) it too
    y = to_dev(y0)
    A.spmv(to_dev(x), y, 1.3, 0.7)
    ref = oracle.csr_spmv(rp, ci, va, x, y0, 1.3, 0.7)
    _, absum = oracle.csr_spmv_f64(rp, ci, va, x, y0, 1.3, 0.7)
    assert_terms_close(to_host(y), ref, absum)


def test_concurrent_spmvs_on_two_streams(sm):
    """SpMVs on one matrix from two streams at once (the reference's AddMatMat only reads
    the object, so concurrent callers are fine there, sparse-matrix.cc:139-194).  The
    multi-slab layout's partial sums and hand-off words belong to the matrix; the library
    orders such SpMVs on the device, so every result equals the one-stream result."""
    torch = torch_dev()
    n_rows, n_cols = 300000, 400000
    rp, ci, va = uniform_csr(n_rows, n_cols, 16, seed=31)
    M = sm.SparseMatrix.from_csr(rp, ci, va, n_cols, opts=dict(layout="bands"))   # AUTO: < 6 M terms, sell
    info = M.info()
    assert info["has_xband"] == 5 and info["xband_slabs"] > 1, info
    rng = np.random.default_rng(32)
    xs = [to_dev(rng.uniform(-1, 1, n_cols).astype(np.float32)) for _ in range(8)]
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    want = [slab_order_for(info, rp, ci, va, to_host(x), y0, 1.0, 0.5)
            for x in xs]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    ys = [to_dev(y0) for _ in xs]
    torch.cuda.synchronize()
    for rep in range(3):
        for i, (x, y) in enumerate(zip(xs, ys)):
            y.copy_(torch.from_numpy(y0).cuda())
        torch.cuda.synchronize()
        for i, (x, y) in enumerate(zip(xs, ys)):
            with torch.cuda.stream(streams[i % 2]):
                M.spmv(x, y, 1.0, 0.5)
        torch.cuda.synchronize()
        for i, y in enumerate(ys):
            assert np.array_equal(bits(to_host(y)), bits(want[i])), (rep, i)
