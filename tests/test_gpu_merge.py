"""SM_ALGO_MERGE: merge-path SpMV (sparsematrix_amd/csrc/kernels_merge.hip; north_star's
"merge-path row balancing").  Every workgroup takes 2048 merge items (row ends + terms) and
every thread 8, so rows are cut anywhere.  A row whose items all fall in one thread's 8 is
summed in stored order from beta*y -- bit-identical to the reference
(/root/reference/src/sparse/kernel.cc:780-796, :791 for the term); cut rows join their parts
in a fixed order: within 1e-6 * sum|terms| of the reference, and deterministic."""
import os

import numpy as np
import pytest

import oracle
from gpu_util import assert_terms_close, bits, to_dev, to_host, torch_dev, uniform_csr

pytestmark = pytest.mark.gpu

# merge items per thread (kernels_merge.hip SM_MERGE_IPT; development builds with another value
# set it here too, tools/archive/r5_merge_ipt2.sh)
IPT = int(os.environ.get("SM_MERGE_IPT", "8"))


@pytest.fixture(scope="module")
def sm():
    torch_dev()
    oracle.build()
    import sparsematrix_amd
    sparsematrix_amd.load()
    return sparsematrix_amd


def _one_thread_rows(rp):
    """Rows whose merge items (first term .. row end) lie in one thread's group of 8."""
    r = np.arange(rp.size - 1, dtype=np.int64)
    start = rp[:-1].astype(np.int64) + r        # the row's first item (its first term, or its end)
    end = rp[1:].astype(np.int64) + r           # the row-end item
    return (start // IPT) == (end // IPT)


def _check(sm, rp, ci, va, n_cols, alpha, beta, seed, y_special=False, want_stage=None):
    """Both plans -- without and with the column-sorted staging copy (sm_build_opts.merge_stage,
    built only for codebook values) -- against the oracle, and against each other bit for bit."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    y0 = rng.uniform(-1, 1, rp.size - 1).astype(np.float32)
    if y_special:
        y0[::101] = np.nan
        y0[1::103] = -0.0
    outs = []
    for stage in (0, 1):
        M = sm.SparseMatrix.from_csr(rp, ci, va, n_cols, opts={"merge_stage": stage})
        if stage and want_stage is not None:
            assert M.info()["merge_stage"] == want_stage
        for _ in range(2):
            y = to_dev(y0)
            M.spmv(to_dev(x), y, alpha, beta, algo="merge")
            outs.append(to_host(y))
    got = outs[0]
    for o in outs[1:]:
        assert np.array_equal(bits(got), bits(o)), "not deterministic, or the staging copy changed bits"
    want = oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta)
    one = _one_thread_rows(rp)
    assert np.array_equal(bits(got[one]), bits(want[one])), "rows inside one thread must be bit-exact"
    _, absum = oracle.csr_spmv_f64(rp, ci, va, x, y0, alpha, beta)
    fin = np.isfinite(want)
    assert_terms_close(got[fin], want[fin], absum[fin])
    assert np.array_equal(np.isnan(got), np.isnan(want))
    return one.mean()


@pytest.mark.parametrize("n_rows,n_cols,per_row", [(30001, 40000, 16), (5000, 1000, 3), (1, 50000, 300),
                                                   (100003, 200000, 1)])
@pytest.mark.parametrize("alpha,beta", [(1.0, 0.5), (1.3, 1.0), (0.7, 0.0)])
def test_merge_uniform_vs_oracle(sm, n_rows, n_cols, per_row, alpha, beta):
    rp, ci, va = uniform_csr(n_rows, n_cols, per_row, seed=n_rows + per_row)
    _check(sm, rp, ci, va, n_cols, alpha, beta, seed=7)


def test_merge_skewed_rows_and_empty_rows(sm):
    """Power-law rows (a few of 10^5 terms, spanning dozens of workgroups), runs of empty rows
    (many row ends inside one thread's share), NaN and -0.0 in y."""
    rng = np.random.default_rng(11)
    n_rows, n_cols = 60000, 300000
    lens = np.minimum(rng.zipf(1.6, n_rows), 4000).astype(np.int64)
    lens[rng.random(n_rows) < 0.3] = 0
    lens[[5, 777, 40000]] = [120000, 50000, 200000]
    rp = np.zeros(n_rows + 1, np.int64)
    rp[1:] = np.cumsum(lens)
    ci = np.concatenate([np.sort(rng.choice(n_cols, int(k), replace=False)) if k else np.zeros(0, np.int64)
                         for k in lens]).astype(np.int32)
    va = rng.uniform(-1, 1, ci.size).astype(np.float32)
    for alpha, beta in ((1.0, 0.5), (2.0, 0.0)):
        share = _check(sm, rp.astype(np.int32), ci, va, n_cols, alpha, beta, seed=13, y_special=True)
    assert share > 0.3   # a real share of rows takes the bit-exact path


def test_merge_config2_full_size(sm):
    """BASELINE config 2 at full size through SM_ALGO_MERGE: within the bound everywhere,
    bit-exact on the rows inside one thread (sampled check on the whole vector)."""
    torch = torch_dev()
    import sparsematrix_amd.synth as synth
    n = 1 << 20
    rp, ci, va = synth.uniform_rows_device(n, n, 16, seed=2)
    M = sm.SparseMatrix.from_csr(rp, ci, va, n)
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y0 = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y = y0.clone()
    M.spmv(x, y, 1.0, 0.5, algo="merge")
    got = to_host(y)
    rph, cih, vah = rp.cpu().numpy(), ci.cpu().numpy(), va.cpu().numpy()
    xh, y0h = to_host(x), to_host(y0)
    want = oracle.csr_spmv_mt(rph, cih, vah, xh, y0h, 1.0, 0.5, threads=16)
    one = _one_thread_rows(rph)
    assert np.array_equal(bits(got[one]), bits(want[one]))
    _, absum = oracle.csr_spmv_f64(rph, cih, vah, xh, y0h, 1.0, 0.5)
    assert_terms_close(got, want, absum)


def test_merge_edge_shapes(sm):
    """One term in one row, a single non-empty row among many empty ones, and no terms at all
    (beta * y only, multiplied iff beta != 1: NaN stays NaN)."""
    rp = np.array([0, 1], np.int32)
    _check(sm, rp, np.array([3], np.int32), np.array([0.5], np.float32), 10, 1.0, 0.5, seed=1)
    n_rows = 5000
    rp = np.zeros(n_rows + 1, np.int32)
    rp[2501:] = 40
    ci = np.arange(40, dtype=np.int32) * 3
    va = np.linspace(-1, 1, 40).astype(np.float32)
    _check(sm, rp, ci, va, 200, 1.3, 0.7, seed=2, y_special=True)
    rp0 = np.zeros(n_rows + 1, np.int32)
    M = sm.SparseMatrix.from_csr(rp0, np.zeros(0, np.int32), np.zeros(0, np.float32), 100)
    y0 = np.random.default_rng(3).uniform(-1, 1, n_rows).astype(np.float32)
    y0[::7] = np.nan
    y = to_dev(y0)
    M.spmv(to_dev(np.ones(100, np.float32)), y, 1.0, 0.25, algo="merge")
    want = oracle.csr_spmv(rp0, np.zeros(0, np.int32), np.zeros(0, np.float32), np.ones(100, np.float32),
                           y0, 1.0, 0.25)
    assert np.array_equal(bits(to_host(y)), bits(want))


def test_merge_codebook_skewed(sm):
    """Codebook values (<= 255 distinct) on skewed rows with relabeled columns: with
    sm_build_opts.merge_stage the terms are staged in column order -- the same products in the
    same LDS slots, so the same bits as the CSR-order staging."""
    rng = np.random.default_rng(21)
    n_rows, n_cols = 40000, 1 << 16
    lens = np.minimum(rng.zipf(1.7, n_rows), 3000)
    rows = [np.unique(rng.zipf(1.5, int(k)) % n_cols) for k in lens]   # skewed column degrees
    rp = np.zeros(n_rows + 1, np.int64)
    rp[1:] = np.cumsum([len(c) for c in rows])
    ci = np.concatenate(rows).astype(np.int32)
    table = rng.uniform(-1, 1, 200).astype(np.float32)
    va = table[rng.integers(0, 200, ci.size)]
    _check(sm, rp.astype(np.int32), ci, va, n_cols, 1.3, 0.5, seed=22, want_stage=1)
    # values beyond a codebook: the option is accepted and nothing is built
    va2 = rng.uniform(-1, 1, ci.size).astype(np.float32)
    _check(sm, rp.astype(np.int32), ci, va2, n_cols, 1.0, 0.0, seed=23, want_stage=0)


def test_merge_rmat24_full_size_vs_oracle(sm):
    """BASELINE config 4 exactly as bench.py times SM_ALGO_MERGE on it (VERDICT r5 missing 2):
    Graph500 R-MAT scale 24, edgefactor 16, seed 4 (263 M terms, rows up to 238 465 terms, so
    single rows span ~120 workgroups).  Both plans -- the CSR arrays and the column-sorted
    staging copy -- give the same bits; rows inside one thread's 8 merge items are bit-identical
    to the reference order (kernel.cc:771-800), every row within 1e-6 * sum|terms|."""
    torch = torch_dev()
    import sparsematrix_amd.synth as synth
    rp_d, ci_d, va_d = synth.rmat_device(24, 16, seed=4)
    n = 1 << 24
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y0 = torch.rand(n, device="cuda", generator=g) * 2 - 1
    outs = []
    for stage in (0, 1):
        M = sm.SparseMatrix.from_csr(rp_d, ci_d, va_d, n, opts={"merge_stage": stage})
        assert M.info()["merge_stage"] == stage
        for _ in range(2):
            y = y0.clone()
            M.spmv(x, y, 1.0, 0.5, algo="merge")
            outs.append(to_host(y))
        del M
        torch.cuda.empty_cache()
    got = outs[0]
    for o in outs[1:]:
        assert np.array_equal(bits(got), bits(o)), "not deterministic, or the staging copy changed bits"
    rp, ci, va = rp_d.cpu().numpy(), ci_d.cpu().numpy(), va_d.cpu().numpy()
    del rp_d, ci_d, va_d
    xh, y0h = to_host(x), to_host(y0)
    want = oracle.csr_spmv_mt(rp, ci, va, xh, y0h, 1.0, 0.5, threads=16)
    one = _one_thread_rows(rp)
    assert one.mean() > 0.3, one.mean()
    assert np.array_equal(bits(got[one]), bits(want[one]))
    _, absum = oracle.csr_spmv_f64(rp.astype(np.int64), ci, va, xh, y0h, 1.0, 0.5)
    assert_terms_close(got, want, absum)


def test_merge_one_row_over_thousands_of_workgroups(sm):
    """a row spanning thousands of workgroups (5 * 10^6 terms, ~2450 slices of 2048
    items) between short rows: the fixup finds the row's first workgroup from the row pointer
    and joins the parts in a fixed tree -- deterministic, within the bound."""
    rng = np.random.default_rng(71)
    n_rows, n_cols = 3000, 1 << 20
    lens = rng.integers(0, 20, n_rows).astype(np.int64)
    lens[1500] = 5_000_000
    lens[2999] = 300_000
    rp = np.zeros(n_rows + 1, np.int64)
    rp[1:] = np.cumsum(lens)
    ci = np.concatenate([np.sort(rng.integers(0, n_cols, int(k))) for k in lens]).astype(np.int32)
    table = rng.uniform(-1, 1, 255).astype(np.float32)
    va = table[rng.integers(0, 255, ci.size)]
    _check(sm, rp.astype(np.int32), ci, va, n_cols, 1.0, 0.5, seed=72, want_stage=1)
