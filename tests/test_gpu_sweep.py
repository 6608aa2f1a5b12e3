"""Column-swept row blocks (sweep.cpp + kernels_sweep.hip) through the C ABI.

One wavefront per 256-row block walks the block's terms in ascending column order,
64-slot chunks with each row's terms in consecutive lanes; a row's partial sums run
through the chunks in column order from beta * y, so every case is compared with the
oracle bit for bit -- ragged and empty rows, rows longer than a chunk, special values,
and BASELINE config 5's column width (2^26 columns, a reduced number of rows)."""
import numpy as np
import pytest

import oracle
from gpu_util import bits, skewed_csr, to_dev, to_host, torch_dev, uniform_csr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sm():
    torch_dev()
    oracle.build()
    import sparsematrix_amd
    sparsematrix_amd.load()
    return sparsematrix_amd


def _sweep(sm, rp, ci, va, n_cols):
    M = sm.SparseMatrix.from_csr(rp, ci, va, n_cols, opts=dict(layout="sweep"))
    info = M.info()
    assert info["sweep_blocks"] == -(-(rp.size - 1) // 256), info
    assert info["has_xband"] == 0 and info["sell_slices"] == 0 and info["ccsell_chunks"] == 0, info
    return M


def _dedup(rp, ci):
    n_rows = rp.size - 1
    row_of = np.repeat(np.arange(n_rows), np.diff(rp))
    keep = np.ones(ci.size, bool)
    keep[1:] = (ci[1:] != ci[:-1]) | (row_of[1:] != row_of[:-1])
    lens = np.bincount(row_of[keep], minlength=n_rows)
    return np.concatenate([[0], np.cumsum(lens)]).astype(np.int32), ci[keep]


@pytest.mark.parametrize("n_rows,n_cols,per_row", [(40000, 300001, 12), (5000, 70000, 40),
                                                   (100001, 1 << 23, 3), (1, 50000, 300),
                                                   (777, 4096, 200)])
def test_sweep_vs_oracle(sm, n_rows, n_cols, per_row):
    rp, ci, va = uniform_csr(n_rows, n_cols, per_row, seed=n_rows + per_row)
    M = _sweep(sm, rp, ci, va, n_cols)
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y0[::97] = np.nan
    for alpha, beta, algo in ((1.0, 1.0, "auto"), (1.3, 0.7, "xband"), (0.5, 0.0, "auto"),
                              (-2.0, 3.0, "auto")):
        y = to_dev(y0)
        M.spmv(to_dev(x), y, alpha, beta, algo=algo)
        want = oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta)
        assert np.array_equal(bits(to_host(y)), bits(want)), (alpha, beta, algo)


def test_sweep_ragged_empty_rows_special_values(sm):
    """Empty rows (beta only), empty blocks, rows of up to 1500 terms (segments across
    many chunks), inf / NaN / -0.0 in the codebook, x and y: bit-exact, signed zeros
    included."""
    rng = np.random.default_rng(9)
    n_rows, n_cols = 30011, 200000
    lengths = np.minimum((rng.pareto(1.2, n_rows) * 5).astype(np.int64), 1500)
    lengths[::5] = 0
    lengths[1024:1536] = 0               # two whole blocks with no terms
    rp, ci, _ = skewed_csr(n_rows, n_cols, lengths, seed=10)
    rp, ci = _dedup(rp, ci)
    table = rng.uniform(-2, 2, 254).astype(np.float32)
    table[:4] = [np.inf, np.nan, -0.0, 0.0]
    va = table[rng.integers(0, table.size, ci.size)]
    M = _sweep(sm, rp, ci, va, n_cols)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    x[0] = np.inf                       # what padding slots point at
    x[7::5003] = np.nan
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y0[:40] = -0.0
    for alpha, beta in ((1.0, 1.0), (1.7, 0.0), (-0.5, 2.0)):
        y = to_dev(y0)
        M.spmv(to_dev(x), y, alpha, beta)
        assert np.array_equal(bits(to_host(y)), bits(oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta)))


def test_sweep_dense_block(sm):
    """Every row of a 300-row block holds all 256 columns: each chunk is one 64-term
    segment, summed lane by lane in column order."""
    n_rows, n_cols = 300, 256
    rp = (np.arange(n_rows + 1) * n_cols).astype(np.int32)
    ci = np.tile(np.arange(n_cols, dtype=np.int32), n_rows)
    rng = np.random.default_rng(11)
    table = rng.uniform(-1, 1, 200).astype(np.float32)
    va = table[rng.integers(0, table.size, ci.size)]
    M = _sweep(sm, rp, ci, va, n_cols)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y = to_dev(y0)
    M.spmv(to_dev(x), y, 0.9, 1.1)
    assert np.array_equal(bits(to_host(y)), bits(oracle.csr_spmv(rp, ci, va, x, y0, 0.9, 1.1)))


def test_sweep_declines_more_than_255_values(sm):
    """More than 255 distinct values: no codebook, the sweep is not built and the matrix
    is still served (bit-exact, the stream kernels)."""
    rp, ci, _ = uniform_csr(3000, 20000, 8, seed=3)
    va = np.random.default_rng(3).uniform(-1, 1, ci.size).astype(np.float32)
    M = sm.SparseMatrix.from_csr(rp, ci, va, 20000, opts=dict(layout="sweep"))
    assert M.info()["sweep_blocks"] == 0
    x = np.random.default_rng(4).uniform(-1, 1, 20000).astype(np.float32)
    y0 = np.zeros(3000, np.float32)
    y = to_dev(y0)
    M.spmv(to_dev(x), y, 1.0, 1.0)
    assert np.array_equal(bits(to_host(y)), bits(oracle.csr_spmv(rp, ci, va, x, y0, 1.0, 1.0)))


def test_sweep_config5_columns_vs_oracle(sm):
    """BASELINE config 5's slice shape at reduced rows: 2^17 rows x 2^26 global columns,
    16 distinct uniform columns per row (seed 5), forced sweep: bit-identical."""
    torch = torch_dev()
    import sparsematrix_amd.synth as synth
    n_rows, n_cols = 1 << 17, 1 << 26
    rp, ci, va = synth.uniform_rows_device(n_rows, n_cols, 16, seed=5)
    S = sm.SparseMatrix.from_csr(rp, ci, va, n_cols, opts=dict(layout="sweep"))
    assert S.info()["sweep_blocks"] == n_rows // 256
    g = torch.Generator(device="cuda").manual_seed(6)
    x = torch.rand(n_cols, device="cuda", generator=g) * 2 - 1
    y0 = torch.rand(n_rows, device="cuda", generator=g) * 2 - 1
    y = y0.clone()
    S.spmv(x, y, 1.0, 0.5)
    rph, cih, vah = rp.cpu().numpy(), ci.cpu().numpy(), va.cpu().numpy()
    want = oracle.csr_spmv_mt(rph, cih, vah, to_host(x), to_host(y0), 1.0, 0.5, threads=16)
    assert np.array_equal(bits(to_host(y)), bits(want))
