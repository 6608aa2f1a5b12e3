"""Device layout builders (sparsematrix_amd/csrc/builddev.hip): from a
device CSR the column relabeling and the sorted sliced ELL are built on the GPU.  Every case
builds the same matrix both ways (sm_build_opts.host_build = 0 / 1) and checks the layouts byte
for byte (sm_layout_digest: relabeling, slice structure, slots, codebook), the reported layout
and the SpMV results bit for bit -- and, for the sliced ELL's rows of <= 2048 terms, the
reference's order (oracle.csr_spmv: kernel.cc:780-796)."""
import time

import numpy as np
import pytest

import oracle
from gpu_util import assert_terms_close, bits, to_host, torch_dev

pytestmark = pytest.mark.gpu

KEYS = ("sell_slices", "sell_codebook", "col_relabel", "n_long_rows", "max_row_nnz", "device_bytes", "has_xband",
        "ccsell_chunks")


@pytest.fixture(scope="module")
def sm():
    torch_dev()
    oracle.build()
    import sparsematrix_amd
    sparsematrix_amd.load()
    return sparsematrix_amd


def _both(sm, rp, ci, va, n_cols, opts=None):
    torch = torch_dev()
    out = []
    for hb in (0, 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        M = sm.SparseMatrix.from_csr(rp, ci, va, n_cols, opts=dict(opts or {}, host_build=hb))
        torch.cuda.synchronize()
        out.append((M, time.perf_counter() - t0))
    (D, td), (H, th) = out
    di, hi = D.info(), H.info()
    assert {k: di[k] for k in KEYS} == {k: hi[k] for k in KEYS}, (di, hi)
    assert D.layout_digest() == H.layout_digest(), (D.layout_digest(), H.layout_digest())
    print(f"build: device {td:.2f} s, host {th:.2f} s", {k: di[k] for k in KEYS[:5]})
    return D, H, di


def _spmv_both(D, H, n_rows, n_cols, seed):
    torch = torch_dev()
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.rand(n_cols, device="cuda", generator=g) * 2 - 1
    y0 = torch.rand(n_rows, device="cuda", generator=g) * 2 - 1
    yd, yh = y0.clone(), y0.clone()
    D.spmv(x, yd, 1.3, 0.5)
    H.spmv(x, yh, 1.3, 0.5)
    assert torch.equal(yd.view(torch.int32), yh.view(torch.int32))
    return to_host(x), to_host(y0), to_host(yd)


def _rmat(scale, seed):
    import sparsematrix_amd.synth as synth
    return synth.rmat_device(scale, 16, seed=seed)


def test_devbuild_rmat18_relabel_codebook_vs_oracle(sm):
    """R-MAT scale 18: relabeled columns, codebook words, rows over 2048 terms cut in
    segments; rows of <= 2048 terms bit-identical to the reference order."""
    rp, ci, va = _rmat(18, 7)
    n = 1 << 18
    D, H, info = _both(sm, rp, ci, va, n, dict(layout="no_bands", relabel=1))   # AUTO: bands here
    assert info["col_relabel"] == 1 and info["sell_codebook"] == 1 and info["sell_slices"] > 0, info
    xh, y0h, got = _spmv_both(D, H, n, n, 3)
    rph, cih, vah = rp.cpu().numpy(), ci.cpu().numpy(), va.cpu().numpy()
    want = oracle.csr_spmv(rph, cih, vah, xh, y0h, 1.3, 0.5)
    short = np.diff(rph.astype(np.int64)) <= 2048
    assert np.array_equal(bits(got[short]), bits(want[short]))
    _, absum = oracle.csr_spmv_f64(rph.astype(np.int64), cih, vah, xh, y0h, 1.3, 0.5)
    assert_terms_close(got, want, absum)


def test_devbuild_plain_values_short_segments(sm):
    """Values beyond a codebook (plain column + value slots), a 64-term segment cap (many long
    rows: sm_build_opts.sell_max_len) and relabeling forced."""
    torch = torch_dev()
    rp, ci, _ = _rmat(16, 9)
    g = torch.Generator(device="cuda").manual_seed(5)
    va = torch.rand(ci.numel(), device="cuda", generator=g) * 2 - 1
    n = 1 << 16
    D, H, info = _both(sm, rp, ci, va, n, dict(layout="no_bands", sell_max_len=64, relabel=1))
    assert info["sell_codebook"] == 0 and info["n_long_rows"] > 0, info
    _spmv_both(D, H, n, n, 4)


def test_devbuild_codebook_edges_and_no_relabel(sm):
    """Exactly 255 and 256 distinct values (codebook / plain), empty rows, and a uniform matrix
    whose relabeling is declined (not skewed): the sliced ELL over the original columns."""
    torch = torch_dev()
    rng = np.random.default_rng(11)
    n_rows, n_cols = 40000, 1 << 20
    lens = rng.integers(0, 40, n_rows)
    lens[::7] = 0
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    ci = np.concatenate([np.sort(rng.choice(n_cols, int(k), replace=False)) for k in lens]).astype(np.int32)
    for k in (255, 256):
        table = rng.uniform(-1, 1, k).astype(np.float32)
        va = table[np.arange(ci.size) % k]   # every value present
        dev = [torch.from_numpy(a).cuda() for a in (rp, ci, va)]
        D, H, info = _both(sm, *dev, n_cols, dict(layout="no_bands"))
        assert info["col_relabel"] == 0 and info["sell_codebook"] == (1 if k == 255 else 0), info
        _spmv_both(D, H, n_rows, n_cols, 6)


def test_devbuild_config4_rmat24_full_size(sm):
    """BASELINE config 4 exactly as bench.py builds it (R-MAT scale 24, seed 4): the device
    build is byte-identical to the host build and much faster (printed)."""
    rp, ci, va = _rmat(24, 4)
    n = 1 << 24
    D, H, info = _both(sm, rp, ci, va, n)
    assert info["col_relabel"] == 1 and info["sell_codebook"] == 1, info
    _spmv_both(D, H, n, n, 8)


# ---- gathered chunk bands (builddev_gcb.hip) -------------------------------------------------
GKEYS = ("has_xband", "xband_slabs", "xband_slab_cols", "device_bytes", "sell_slices", "col_relabel")


def _both_gcb(sm, rp, ci, va, n_cols, opts):
    """Device and host builds of one CSR (device tensors): same layout bytes and info."""
    torch = torch_dev()
    dev = [a if hasattr(a, "device") else torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (rp, ci, va)]
    out = []
    for hb in (0, 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        M = sm.SparseMatrix.from_csr(*dev, n_cols, opts=dict(opts, host_build=hb))
        torch.cuda.synchronize()
        out.append((M, time.perf_counter() - t0))
    (D, td), (H, th) = out
    di, hi = D.info(), H.info()
    assert {k: di[k] for k in GKEYS} == {k: hi[k] for k in GKEYS}, (di, hi)
    assert D.layout_digest() == H.layout_digest(), (D.layout_digest(), H.layout_digest())
    print(f"gcb build: device {td:.2f} s, host {th:.2f} s", {k: di[k] for k in GKEYS[:3]})
    return D, H, di, td, th


def _gcb_spmv_check(D, H, info, rp, ci, va, n_rows, n_cols, seed):
    x = np.random.default_rng(seed).uniform(-1, 1, n_cols).astype(np.float32)
    y0 = np.random.default_rng(seed + 1).uniform(-1, 1, n_rows).astype(np.float32)
    torch = torch_dev()
    yd, yh = torch.from_numpy(y0).cuda(), torch.from_numpy(y0).cuda()
    xd = torch.from_numpy(x).cuda()
    D.spmv(xd, yd, 1.3, 0.5)
    H.spmv(xd, yh, 1.3, 0.5)
    assert torch.equal(yd.view(torch.int32), yh.view(torch.int32))
    if info["has_xband"] == 6 and info["xband_slabs"] == 1:   # one slab: the reference's order
        want = oracle.csr_spmv(rp, ci, va, x, y0, 1.3, 0.5)
        assert np.array_equal(bits(to_host(yd)), bits(want))


@pytest.mark.parametrize("n_rows,n_cols,per_row", [(200003, 3000001, 16), (9000, 70001, 40), (5000, 1000, 5),
                                                   (1, 50000, 30), (300000, 8000000, 4)])
@pytest.mark.parametrize("slabs", [1, 0, 3])
def test_devbuild_gcb_uniform(sm, n_rows, n_cols, per_row, slabs):
    """Forced gcb on uniform shapes (test_gpu_gcb.py's), one, AUTO's and three slabs: the device
    build's bands byte-identical to gcb.cpp's, the SpMV bit-identical (and with one slab the
    reference's order)."""
    from gpu_util import uniform_csr
    rp, ci, va = uniform_csr(n_rows, n_cols, per_row, seed=n_rows + n_cols)
    D, H, info, _, _ = _both_gcb(sm, rp, ci, va, n_cols, dict(layout="gcb", band_slabs=slabs))
    assert info["has_xband"] == 6, info
    _gcb_spmv_check(D, H, info, rp, ci, va, n_rows, n_cols, 3)


def test_devbuild_gcb_long_segments_hub_columns(sm):
    """Rows of 90 consecutive columns (cut inside the run: a band holds at most 63 terms of a
    row), two hub columns in every row (a column's rows split over several bands)."""
    rng = np.random.default_rng(3)
    n_rows, n_cols, w = 6000, 700000, 90
    rows = [np.union1d(np.arange(s, s + w), [5, 600000]) for s in rng.integers(0, n_cols - w - 10, n_rows)]
    rp = np.zeros(n_rows + 1, np.int32)
    rp[1:] = np.cumsum([len(c) for c in rows])
    ci = np.concatenate(rows).astype(np.int32)
    va = rng.uniform(-1, 1, ci.size).astype(np.float32)
    for slabs in (1, 0):
        D, H, info, _, _ = _both_gcb(sm, rp, ci, va, n_cols, dict(layout="gcb", band_slabs=slabs))
        assert info["has_xband"] == 6, info
        _gcb_spmv_check(D, H, info, rp, ci, va, n_rows, n_cols, 4)


def test_devbuild_gcb_ragged_and_declines(sm):
    """Empty rows, a 3000-term row, empty column ranges, a partial last block; and a row whose
    columns are not ascending, which both builders decline (the same fallback layout)."""
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
    D, H, info, _, _ = _both_gcb(sm, rp, ci, va, n_cols, dict(layout="gcb", band_slabs=1))
    assert info["has_xband"] == 6 and info["xband_slabs"] == 1, info
    _gcb_spmv_check(D, H, info, rp, ci, va, n_rows, n_cols, 5)
    ci2 = ci.copy()
    a = int(rp[777])   # the 3000-term row: swap its first two columns
    ci2[a], ci2[a + 1] = ci2[a + 1], ci2[a]
    D2, H2, info2, _, _ = _both_gcb(sm, rp, ci2, va, n_cols, dict(layout="gcb", band_slabs=1))
    assert info2["has_xband"] != 6, info2


def test_devbuild_gcb_config5_rank0_slice(sm):
    """Config 5's rank-0 slice as bench.py builds it (2^23 rows x 2^26 columns, 16 per row,
    seed 5), AUTO: the device build byte-identical to the host's, under 1.5 s, the SpMV the
    same bits."""
    import sparsematrix_amd.synth as synth
    n_rows, n_cols = 1 << 23, 1 << 26
    rp, ci, va = synth.uniform_rows_device(n_rows, n_cols, 16, seed=5)
    D, H, info, td, th = _both_gcb(sm, rp, ci, va, n_cols, {})
    assert info["has_xband"] == 6, info
    torch = torch_dev()
    g = torch.Generator(device="cuda").manual_seed(6)
    x = torch.rand(n_cols, device="cuda", generator=g) * 2 - 1
    y0 = torch.rand(n_rows, device="cuda", generator=g) * 2 - 1
    yd, yh = y0.clone(), y0.clone()
    D.spmv(x, yd, 1.0, 0.5)
    H.spmv(x, yh, 1.0, 0.5)
    assert torch.equal(yd.view(torch.int32), yh.view(torch.int32))
    assert td < 1.5, (td, th)


# ---- the merge path's staging copy (builddev.hip devbuild_merge_stage) ----------------------
def test_devbuild_merge_stage_rmat_relabeled_and_plain(sm):
    """sm_build_opts.merge_stage on a device CSR: R-MAT 18 (relabeled columns, codebook) and a
    uniform matrix without relabeling -- the staging words, offsets and table byte-identical to
    merge_stage_build's (digest [3]), SM_ALGO_MERGE the same bits either way."""
    torch = torch_dev()
    from gpu_util import uniform_csr
    rp, ci, va = _rmat(18, 7)
    cases = [(rp, ci, va, 1 << 18, 1 << 18, dict(layout="no_bands", relabel=1, merge_stage=1))]
    r2, c2, v2 = uniform_csr(70000, 90000, 12, seed=4)
    cases.append(tuple(torch.from_numpy(a).cuda() for a in (r2, c2, v2)) + (70000, 90000, dict(merge_stage=1)))
    for rp_, ci_, va_, n_rows, n_cols, opts in cases:
        D, H, info = _both(sm, rp_, ci_, va_, n_cols, opts)
        assert info["merge_stage"] == 1 and D.layout_digest()[3] != 0, info
        g = torch.Generator(device="cuda").manual_seed(9)
        x = torch.rand(n_cols, device="cuda", generator=g) * 2 - 1
        y0 = torch.rand(n_rows, device="cuda", generator=g) * 2 - 1
        yd, yh = y0.clone(), y0.clone()
        D.spmv(x, yd, 1.3, 0.5, algo="merge")
        H.spmv(x, yh, 1.3, 0.5, algo="merge")
        assert torch.equal(yd.view(torch.int32), yh.view(torch.int32))


def test_devbuild_merge_stage_declines_beyond_codebook(sm):
    """More than 255 distinct values: both builders decline the staging copy."""
    torch = torch_dev()
    rp, ci, _ = _rmat(14, 3)
    g = torch.Generator(device="cuda").manual_seed(2)
    va = torch.rand(ci.numel(), device="cuda", generator=g)
    D, H, info = _both(sm, rp, ci, va, 1 << 14, dict(layout="no_bands", merge_stage=1))
    assert info["merge_stage"] == 0, info


def test_device_csr_validation_flags(sm):
    """sm_create_from_csr_device rejects what the host path rejects (validate_kernel: row
    pointers start at 0, end at nnz, never decrease; columns in range) -- including a bad
    column deep inside one long row -- and accepts the repaired arrays."""
    torch = torch_dev()
    rng = np.random.default_rng(4)
    n_rows, n_cols = 5000, 3000
    lens = rng.integers(0, 9, n_rows)
    lens[1234] = 2500
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    ci = np.concatenate([np.sort(rng.choice(n_cols, int(k), replace=False)) for k in lens]).astype(np.int32)
    va = rng.uniform(-1, 1, ci.size).astype(np.float32)

    def build(r, c):
        dev = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (r, c, va)]
        return sm.SparseMatrix.from_csr(*dev, n_cols)

    build(rp, ci)   # valid
    bad_col = ci.copy()
    bad_col[rp[1234] + 2000] = n_cols
    neg_col = ci.copy()
    neg_col[-1] = -1
    bad_first = rp.copy()
    bad_first[0] = 1
    bad_last = rp.copy()
    bad_last[-1] -= 1
    bad_order = rp.copy()
    bad_order[100], bad_order[101] = bad_order[101] + 1, bad_order[100]
    for r, c in ((rp, bad_col), (rp, neg_col), (bad_first, ci), (bad_last, ci), (bad_order, ci)):
        with pytest.raises(sm.SparseMatrixError):
            build(r, c)
