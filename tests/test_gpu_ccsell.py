"""Column-chunked sorted sliced-ELL SpMV (ccsell.cpp + kernels_ccsell.hip) through the C ABI.

One launch per column chunk, in chunk order; each lane adds its row's terms of that
chunk to y[row] in stored order, the row's first unit applying beta: every row is
summed in the reference's order (ascending column), so every case is compared with
the oracle bit for bit -- including BASELINE config 5's column width (2^26 columns,
a reduced number of rows)."""
import numpy as np
import pytest

import oracle
from gpu_util import assert_terms_close, bits, skewed_csr, to_dev, to_host, torch_dev, uniform_csr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sm():
    torch_dev()
    oracle.build()
    import sparsematrix_amd
    sparsematrix_amd.load()
    return sparsematrix_amd


def _cc(sm, rp, ci, va, n_cols, chunk_log2, codebook=True):
    M = sm.SparseMatrix.from_csr(rp, ci, va, n_cols,
                                 opts=dict(layout="no_bands", ccsell=1, ccsell_chunk_log2=chunk_log2,
                                           sell_codebook=-1 if codebook else 0))
    info = M.info()
    assert info["ccsell_chunks"] == -(-n_cols // (1 << chunk_log2)), info
    assert info["sell_slices"] == 0 and info["has_xband"] == 0, info
    return M, info


@pytest.mark.parametrize("n_rows,n_cols,per_row,chunk_log2", [(40000, 300001, 12, 14),
                                                               (5000, 70000, 40, 12),
                                                               (100000, 1 << 20, 3, 16),
                                                               (1, 50000, 300, 10)])
@pytest.mark.parametrize("codebook", [True, False])
def test_ccsell_vs_oracle(sm, n_rows, n_cols, per_row, chunk_log2, codebook):
    rp, ci, va = uniform_csr(n_rows, n_cols, per_row, seed=n_rows + chunk_log2)
    if not codebook:
        va = np.random.default_rng(3).uniform(-1, 1, va.size).astype(np.float32)
    M, info = _cc(sm, rp, ci, va, n_cols, chunk_log2, codebook)
    assert info["sell_codebook"] == int(codebook)
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y0[::97] = np.nan
    for alpha, beta, algo in ((1.0, 1.0, "auto"), (1.3, 0.7, "sell"), (0.5, 0.0, "auto"),
                              (-2.0, 3.0, "xband")):
        y = to_dev(y0)
        M.spmv(to_dev(x), y, alpha, beta, algo=algo)
        want = oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta)
        assert np.array_equal(bits(to_host(y)), bits(want)), (alpha, beta, algo)


def test_ccsell_ragged_empty_rows_special_values(sm):
    """Empty rows (beta only), rows spanning many chunks, inf / NaN / -0.0 in values, x
    and y: bit-exact, signed zeros included."""
    rng = np.random.default_rng(9)
    n_rows, n_cols = 30011, 200000
    lengths = np.minimum((rng.pareto(1.2, n_rows) * 5).astype(np.int64), 1500)
    lengths[::5] = 0
    rp, ci, _ = skewed_csr(n_rows, n_cols, lengths, seed=10)
    # skewed_csr allows repeated columns; ccsell needs strictly ascending rows
    row_of = np.repeat(np.arange(n_rows), np.diff(rp))
    keep = np.ones(ci.size, bool)
    keep[1:] = (ci[1:] != ci[:-1]) | (row_of[1:] != row_of[:-1])
    lens = np.bincount(row_of[keep], minlength=n_rows)
    ci = ci[keep]
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    table = rng.uniform(-2, 2, 200).astype(np.float32)
    table[:4] = [np.inf, np.nan, -0.0, 0.0]
    va = table[rng.integers(0, table.size, ci.size)]
    M, _ = _cc(sm, rp, ci, va, n_cols, 13)
    x = rng.uniform(-1, 1, n_cols).astype(np.float32)
    x[0] = np.inf                       # what padding words point at
    x[7::5003] = np.nan
    y0 = rng.uniform(-1, 1, n_rows).astype(np.float32)
    y0[:40] = -0.0
    for alpha, beta in ((1.0, 1.0), (1.7, 0.0), (-0.5, 2.0)):
        y = to_dev(y0)
        M.spmv(to_dev(x), y, alpha, beta)
        assert np.array_equal(bits(to_host(y)), bits(oracle.csr_spmv(rp, ci, va, x, y0, alpha, beta)))


def test_ccsell_declines_long_run_in_one_chunk(sm):
    """A row with more than 2048 terms inside one column chunk: ccsell declines and the
    sliced ELL serves the matrix (rows > 2048 terms as segments, within the bound)."""
    n_cols = 1 << 20
    ci = np.arange(0, 3000, dtype=np.int32)
    rp = np.array([0, 3000, 3001], np.int32)
    ci = np.concatenate([ci, [5]]).astype(np.int32)
    va = np.ones(ci.size, np.float32)
    M = sm.SparseMatrix.from_csr(rp, ci, va, n_cols, opts=dict(ccsell=1))
    info = M.info()
    assert info["ccsell_chunks"] == 0 and info["sell_slices"] > 0, info


def test_config5_columns_auto_ccsell_vs_oracle(sm):
    """BASELINE config 5's slice shape at reduced rows: 2^17 rows x 2^26 global columns,
    16 distinct uniform columns per row (seed 5).  The column-chunked layout (x = 256 MiB,
    64 chunks of 4 MiB; forced here) is bit-identical to the oracle on every row; AUTO
    (the gather-band kind by its cost model, capi.cpp gather_cost_ok) is bit-identical with
    one slab and within 1e-6 * sum|terms| with several (slab sums added in slab order)."""
    torch = torch_dev()
    import sparsematrix_amd.synth as synth
    n_rows, n_cols = 1 << 17, 1 << 26
    rp, ci, va = synth.uniform_rows_device(n_rows, n_cols, 16, seed=5)
    C = sm.SparseMatrix.from_csr(rp, ci, va, n_cols, opts=dict(layout="no_bands", ccsell=1))
    info = C.info()
    assert info["ccsell_chunks"] == 64 and info["has_xband"] == 0, info
    A = sm.SparseMatrix.from_csr(rp, ci, va, n_cols)
    ainfo = A.info()
    assert ainfo["has_xband"] in (3, 6) or ainfo["ccsell_chunks"] > 0, ainfo
    g = torch.Generator(device="cuda").manual_seed(6)
    x = torch.rand(n_cols, device="cuda", generator=g) * 2 - 1
    y0 = torch.rand(n_rows, device="cuda", generator=g) * 2 - 1
    y, ya = y0.clone(), y0.clone()
    C.spmv(x, y, 1.0, 0.5)
    A.spmv(x, ya, 1.0, 0.5)
    rph, cih, vah = rp.cpu().numpy(), ci.cpu().numpy(), va.cpu().numpy()
    want = oracle.csr_spmv_mt(rph, cih, vah, to_host(x), to_host(y0), 1.0, 0.5, threads=16)
    assert np.array_equal(bits(to_host(y)), bits(want))
    if ainfo["has_xband"] == 0 or ainfo["xband_slabs"] == 1:
        assert np.array_equal(bits(to_host(ya)), bits(want))
    else:
        _, absum = oracle.csr_spmv_f64(rph.astype(np.int64), cih, vah, to_host(x), to_host(y0), 1.0, 0.5)
        assert_terms_close(to_host(ya), want, absum)


def test_config5_rank0_slice_full_size_auto_vs_oracle(sm):
    """the slice bench.py times for config 5 (`--workload config5
    --emulate-world 8`, and rank 0 of the 8-GPU run): rank 0's FULL 2^23 rows x 2^26 global
    columns, 16 distinct uniform columns per row, seed 5 (bench.py: seed0 + 1000 k +
    7919 rank), AUTO.  AUTO must build the gathered chunk bands (has_xband == 6, gcb) the bench
    measures; its SpMV is compared with the oracle's same-order CSR SpMV over all 2^23
    rows: bit for bit with one slab (rows summed in the reference's order), within
    1e-6 * sum|terms| with several (slab sums in slab order)."""
    torch = torch_dev()
    import sparsematrix_amd.synth as synth
    n_rows, n_cols = 1 << 23, 1 << 26
    rp, ci, va = synth.uniform_rows_device(n_rows, n_cols, 16, seed=5)
    A = sm.SparseMatrix.from_csr(rp, ci, va, n_cols)
    info = A.info()
    assert info["has_xband"] == 6, info          # gathered chunk bands, as bench.py reports
    g = torch.Generator(device="cuda").manual_seed(6)
    x = torch.rand(n_cols, device="cuda", generator=g) * 2 - 1
    y0 = torch.rand(n_rows, device="cuda", generator=g) * 2 - 1
    y = y0.clone()
    A.spmv(x, y, 1.0, 0.5)
    y2 = y0.clone()
    A.spmv(x, y2, 1.0, 0.5)                      # deterministic: a second launch, same bits
    got, got2 = to_host(y), to_host(y2)
    assert np.array_equal(bits(got), bits(got2))
    rph, cih, vah = rp.cpu().numpy(), ci.cpu().numpy(), va.cpu().numpy()
    del rp, ci, va
    xh, y0h = to_host(x), to_host(y0)
    want = oracle.csr_spmv_mt(rph, cih, vah, xh, y0h, 1.0, 0.5, threads=16)
    if info["xband_slabs"] == 1:
        assert np.array_equal(bits(got), bits(want))
    else:
        _, absum = oracle.csr_spmv_f64(rph.astype(np.int64), cih, vah, xh, y0h, 1.0, 0.5)
        assert_terms_close(got, want, absum)
