"""SM_ALGO_MFMA: the SpMM with N = 32 right-hand sides on the matrix cores
(sparsematrix_amd/csrc/spmm_mfma.hip; VERDICT r3 item 8, north_star's "MFMA used only on
the dense N-panel of SpMM").  Not bit-identical to the reference (one fused rounding per
term): checked within 1e-6 * sum|terms| against the oracle's same-order SpMM
(oracle.csr_spmm, /root/reference/src/sparse/kernel.cc:568-582), and bit for bit against
the fma-chain model of the matrix cores' arithmetic (oracle.csr_spmm_fma, test-only)."""
import numpy as np
import pytest

import oracle
from gpu_util import assert_terms_close, bits, to_dev, to_host, torch_dev, uniform_csr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sm():
    torch_dev()
    oracle.build()
    import sparsematrix_amd
    sparsematrix_amd.load()
    return sparsematrix_amd


def _absum_spmm(rp, ci, va, X, Y0, alpha, beta):
    """Per output: |beta*y| + sum |alpha*v*x| (fp64), column by column."""
    ab = np.empty(Y0.shape, np.float64)
    for j in range(X.shape[1]):
        _, a = oracle.csr_spmv_f64(rp.astype(np.int64), ci, va, np.ascontiguousarray(X[:, j]),
                                   np.ascontiguousarray(Y0[:, j]), alpha, beta)
        ab[:, j] = a
    return ab


def _ragged(n_rows, n_cols, seed):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 40, n_rows)
    lens[rng.random(n_rows) < 0.1] = 0                 # empty rows
    lens[rng.integers(0, n_rows, 3)] = 700              # a few long rows
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    ci = np.concatenate([np.sort(rng.choice(n_cols, l, replace=False)) for l in lens]).astype(np.int32)
    va = rng.uniform(-1, 1, ci.size).astype(np.float32)
    return rp, ci, va


@pytest.mark.parametrize("shape", ["uniform", "ragged"])
@pytest.mark.parametrize("alpha,beta", [(1.0, 0.5), (1.3, 1.0), (-0.7, 0.0)])
def test_spmm_mfma_vs_oracle(sm, shape, alpha, beta):
    if shape == "uniform":
        n_rows, n_cols = 30001, 40000            # not a multiple of 16: a partial last tile
        rp, ci, va = uniform_csr(n_rows, n_cols, 16, seed=31)
    else:
        n_rows, n_cols = 5003, 9000
        rp, ci, va = _ragged(n_rows, n_cols, 32)
    M = sm.SparseMatrix.from_csr(rp, ci, va, n_cols)
    rng = np.random.default_rng(33)
    X = rng.uniform(-1, 1, (n_cols, 32)).astype(np.float32)
    Y0 = rng.uniform(-1, 1, (M.n_rows, 32)).astype(np.float32)
    Y = to_dev(Y0)
    M.spmm(to_dev(X), Y, alpha, beta, algo="mfma")
    got = to_host(Y)
    want = oracle.csr_spmm(rp.astype(np.int64), ci, va, X, Y0, alpha, beta)
    assert_terms_close(got, want, _absum_spmm(rp, ci, va, X, Y0, alpha, beta))
    model = oracle.csr_spmm_fma(rp.astype(np.int64), ci, va, X, Y0, alpha, beta)
    assert np.array_equal(_zero_sign_free(got), _zero_sign_free(model))


def _zero_sign_free(a):
    """Bits with -0.0 read as +0.0: a tile's other rows' zero A entries add fma(0, x, acc),
    which turns an accumulator of -0.0 (beta = 0 on a negative y, an empty row) into +0.0;
    every other value is the fma chain's exactly."""
    b = bits(a).copy()
    b[b == 0x80000000] = 0
    return b


def test_spmm_mfma_config3_full_size(sm):
    """Config 3 at full size: 2^20 x 2^20, 16 terms per row, N = 32 (seed 2 matrix, seed 3
    panel as bench.py); within the bound on every output and equal to the fma-chain model."""
    torch = torch_dev()
    import sparsematrix_amd.synth as synth
    n = 1 << 20
    rp, ci, va = synth.uniform_rows_device(n, n, 16, seed=2)
    M = sm.SparseMatrix.from_csr(rp, ci, va, n)
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.rand((n, 32), generator=g, device="cuda") * 2 - 1
    Y0 = torch.rand((n, 32), generator=g, device="cuda") * 2 - 1
    Y = Y0.clone()
    M.spmm(X, Y, 1.0, 0.5, algo="mfma")
    got = to_host(Y)
    rph, cih, vah = rp.cpu().numpy().astype(np.int64), ci.cpu().numpy(), va.cpu().numpy()
    Xh, Y0h = to_host(X), to_host(Y0)
    model = oracle.csr_spmm_fma(rph, cih, vah, Xh, Y0h, 1.0, 0.5)
    assert np.array_equal(bits(got), bits(model))
    want = oracle.csr_spmm(rph, cih, vah, Xh, Y0h, 1.0, 0.5)
    rows = np.random.default_rng(4).choice(n, 4096, replace=False)   # sampled bound check
    sub = np.zeros(n + 1, np.int64)
    ab = np.empty((rows.size, 32))
    for j in range(32):
        _, a = oracle.csr_spmv_f64(rph, cih, vah, np.ascontiguousarray(Xh[:, j]),
                                   np.ascontiguousarray(Y0h[:, j]), 1.0, 0.5)
        ab[:, j] = a[rows]
    del sub
    assert_terms_close(got[rows], want[rows], ab)


def test_spmm_mfma_rejects_other_shapes(sm):
    from sparsematrix_amd import _lib
    rp, ci, va = uniform_csr(100, 200, 4, seed=1)
    M = sm.SparseMatrix.from_csr(rp, ci, va, 200)
    X = to_dev(np.ones((200, 16), np.float32))
    Y = to_dev(np.ones((100, 16), np.float32))
    with pytest.raises(_lib.SparseMatrixError):
        M.spmm(X, Y, 1.0, 1.0, algo="mfma")
    with pytest.raises(_lib.SparseMatrixError):
        M.spmv(to_dev(np.ones(200, np.float32)), to_dev(np.ones(100, np.float32)), algo="mfma")
