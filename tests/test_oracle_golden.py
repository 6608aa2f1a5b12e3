"""Pin the C restatement (oracle/refmodel.c) against the reference's own outputs.

CPU only.  Every committed fixture (tests/golden, produced by the real reference)
must be reproduced bit-for-bit: encoded stream (positions, ids, panel bounds),
CopyTo, AddMatMat, and the same-order CSR kernels derived from the stream.
"""
import numpy as np
import pytest

import oracle
from golden_util import bits_equal, case_names, load_case, load_kernels


@pytest.fixture(scope="module", autouse=True)
def _built():
    oracle.build()


@pytest.mark.parametrize("name", case_names())
def test_encode_stream_bit_exact(name):
    c = load_case(name)
    om = oracle.RefModel(c.dm, c.rows, c.cols, c.stride, c.table, c.table_size, c.trans)
    st = om.stream()
    assert (st.rows, st.cols) == (c.s_rows, c.s_cols)
    assert np.array_equal(st.pos, c.pos)
    assert np.array_equal(st.val, c.val)
    assert np.array_equal(st.panel_row_off, c.panel_row_off)
    assert np.array_equal(st.panel_col_off, c.panel_col_off)
    assert np.array_equal(st.panel_begin, c.panel_begin)
    assert np.array_equal(st.panel_end, c.panel_end)


@pytest.mark.parametrize("name", case_names())
def test_copyto_bit_exact(name):
    c = load_case(name)
    om = oracle.RefModel(c.dm, c.rows, c.cols, c.stride, c.table, c.table_size, c.trans)
    if c.copyto:
        for tr, (stride, want) in c.copyto.items():
            assert bits_equal(om.copy_to(stride, tr), want)
    # index rule (covers the large cases whose CopyTo is not stored)
    got = om.copy_to(c.s_rows, True).reshape(c.s_cols, c.s_rows)
    assert bits_equal(got, c.dense_b())


@pytest.mark.parametrize("name", case_names())
def test_addmatmat_bit_exact(name):
    c = load_case(name)
    om = oracle.RefModel(c.dm, c.rows, c.cols, c.stride, c.table, c.table_size, c.trans)
    assert c.runs
    for r in c.runs:
        out = om.add_mat_mat(r.a, r.m, r.lda, r.c, r.ldc, r.alpha, r.beta)
        assert bits_equal(out, r.out), (r.m, r.alpha, r.beta)


@pytest.mark.parametrize("name", case_names())
def test_same_order_csr_bit_exact(name):
    """CSR(B) SpMV / SpMM with the reference's op order reproduce AddMatMat exactly."""
    c = load_case(name)
    om = oracle.RefModel(c.dm, c.rows, c.cols, c.stride, c.table, c.table_size, c.trans)
    rp, ci, va, td = om.to_csr()
    k, n = c.s_rows, c.s_cols
    assert rp[-1] == int(c.live_mask_b().sum())
    for r in c.runs:
        A = r.a.reshape(r.m, r.lda)[:, :k]
        Cin = r.c.reshape(r.m, r.ldc)
        want = r.out.reshape(r.m, r.ldc)
        if r.m == 1:
            y = oracle.csr_spmv(rp, ci, va, A[0], Cin[0, :n], r.alpha, r.beta)
            assert bits_equal(y, want[0, :n])
        Y = oracle.csr_spmm(rp, ci, va, np.ascontiguousarray(A.T), np.ascontiguousarray(Cin[:, :n].T),
                            r.alpha, r.beta)
        assert bits_equal(Y.T, want[:, :n])
        # columns past n are untouched
        assert bits_equal(want[:, n:], Cin[:, n:])


def test_selftest_kat_values():
    """sparse-matrix.cc:220-226: CopyTo = {1.1,0,0,4.4,8.8,0}; c = {92.513, 44.6} (1e-3)."""
    for name in ("kat_selftest_notrans", "kat_selftest_trans"):
        c = load_case(name)
        om = oracle.RefModel(c.dm, c.rows, c.cols, c.stride, c.table, c.table_size, c.trans)
        got = om.copy_to(2, False)
        assert np.array_equal(got, np.array([1.1, 0, 0, 4.4, 8.8, 0], np.float32))
        r = c.runs[0]
        out = om.add_mat_mat(r.a, 1, 3, r.c, 2, 1.3, 2.0)
        assert abs(out[0] - 92.513) <= 1e-3 and abs(out[1] - 44.6) <= 1e-3


def test_kernel_helpers_bit_exact():
    k = load_kernels()
    got = oracle.beta_scale(k["beta_c"], int(k["beta_m"]), int(k["beta_n"]), int(k["beta_ldc"]),
                            float(k["beta"]))
    assert bits_equal(got, k["beta_out"])
    tm, tn, lda, ldsa = (int(k[x]) for x in ("trans_m", "trans_n", "trans_lda", "trans_ldsa"))
    got = oracle.transpose(k["trans_a"], tm, tn, lda, ldsa, tn * ldsa)
    want = k["trans_out"].reshape(tn, ldsa)[:, :tm]
    assert bits_equal(got.reshape(tn, ldsa)[:, :tm], want)


@pytest.mark.skipif(not oracle.ref_available(), reason="reference build only in the dev container")
def test_restatement_vs_live_reference_random():
    """Extra random cases against the compiled reference (dev container only)."""
    rng = np.random.default_rng(12345)
    for _ in range(40):
        rows, cols = (int(x) for x in rng.integers(1, 600, 2))
        stride = cols + int(rng.integers(0, 3))
        dens = float(rng.choice([0.0005, 0.01, 0.3]))
        T = int(rng.integers(1, 256))
        trans = bool(rng.integers(0, 2))
        dm = np.full(rows * stride, 255, np.uint8)
        live = rng.random(rows * stride) < dens
        dm[live] = rng.integers(0, 255, int(live.sum()))
        table = rng.uniform(-1, 1, 255).astype(np.float32)
        ref = oracle.Reference(dm, rows, cols, stride, table, T, trans)
        om = oracle.RefModel(dm, rows, cols, stride, table, T, trans)
        a_s, o_s = ref.stream(), om.stream()
        assert np.array_equal(a_s.pos, o_s.pos) and np.array_equal(a_s.val, o_s.val)
        m = int(rng.integers(1, 20))
        kk, nn = om.rows, om.cols
        a = rng.uniform(-1e3, 1e3, m * kk + 1).astype(np.float32)
        cc = rng.uniform(-1e3, 1e3, m * nn + 1).astype(np.float32)
        al, be = float(rng.choice([1.0, 1.3, 0.0])), float(rng.choice([1.0, 0.7, 0.0]))
        assert bits_equal(ref.add_mat_mat(a, m, kk, cc, nn, al, be),
                          om.add_mat_mat(a, m, kk, cc, nn, al, be))


def test_csr_spmv_multithread_bit_identical():
    """The all-cores CPU baseline (OpenMP rows) sums every row in the same order."""
    rng = np.random.default_rng(11)
    n, per = 50000, 16
    rp = np.arange(0, n * per + 1, per, dtype=np.int32)
    ci = np.sort(rng.integers(0, n, (n, per)), 1).astype(np.int32).ravel()
    va = rng.uniform(-1, 1, n * per).astype(np.float32)
    x = rng.uniform(-1, 1, n).astype(np.float32)
    y = rng.uniform(-1, 1, n).astype(np.float32)
    want = oracle.csr_spmv(rp, ci, va, x, y, 1.3, 0.7)
    for t in (1, 3, 8):
        got = oracle.csr_spmv_mt(rp, ci, va, x, y, 1.3, 0.7, threads=t)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), t
