"""CPU-side checks of the drop-in boundary (no GPU compute).

The C-ABI library must build for gfx950, load, export every entry point that
include/sparsematrix.h declares, and fail loudly (SM_ERR_NO_DEVICE) instead of
computing anything on the host when no GPU is visible.
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sparsematrix.h")


@pytest.fixture(scope="module")
def lib():
    subprocess.run(["make", "-s", "-C", ROOT, "-j", "8"], check=True)
    from sparsematrix_amd import _lib
    return _lib.load()


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"SM_API[^;(]*?\b(sm_\w+)\s*\(", text, flags=re.S)))


def test_header_declares_expected_api():
    from sparsematrix_amd import _lib
    assert declared_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "sparsematrix_amd",
                                                                     "libsparsematrix_amd.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (\w+)$", out, flags=re.M))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    for s in declared_symbols():
        assert hasattr(lib, s)


def test_library_is_gfx950(lib):
    so = os.path.join(ROOT, "sparsematrix_amd", "libsparsematrix_amd.so")
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          f"--input={so}"], capture_output=True, text=True)
    text = out.stdout + out.stderr
    if "gfx" not in text:   # bundle may sit in .hip_fatbin; fall back to strings
        text = subprocess.run(["strings", so], capture_output=True, text=True).stdout
    assert "gfx950" in text


def test_status_strings(lib):
    assert b"gfx950" in lib.sm_version()
    for s in range(8):
        assert lib.sm_status_string(s)


def test_no_host_fallback_without_gpu(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    n = C.c_int32(-1)
    assert lib.sm_device_count(C.byref(n)) == 7 and n.value == 0
    import sparsematrix_amd as smd
    with pytest.raises(smd.SparseMatrixError) as ei:
        smd.SparseMatrix(np.zeros(4, np.uint8), 2, 2, 2, np.ones(1, np.float32), 1)
    assert ei.value.status == 7
    with pytest.raises(smd.SparseMatrixError):
        smd.SparseMatrix.from_csr(np.array([0, 1], np.int32), np.array([0], np.int32),
                                  np.ones(1, np.float32), 1)


def test_argument_validation_without_gpu(lib):
    h = C.c_void_p()
    # table_size out of range is rejected before any device work (sparse-matrix.cc:25)
    assert lib.sm_create_from_dense_index(None, 1, 1, 1, None, 256, 0, 0, C.byref(h)) == 1
    assert lib.sm_create_from_csr(-1, 1, 0, None, None, None, 0, C.byref(h)) == 1
    assert lib.sm_create_from_csr(1 << 31, 1, 0, None, None, None, 0, C.byref(h)) == 5
    bad_rp = np.array([0, 2, 1], np.int32)
    ci = np.zeros(2, np.int32)
    va = np.zeros(2, np.float32)
    assert lib.sm_create_from_csr(2, 4, 1, bad_rp.ctypes.data, ci.ctypes.data, va.ctypes.data, 0,
                                  C.byref(h)) == 6
    assert lib.sm_spmv(None, 1.0, None, 1.0, None, 0, None) == 1
    from sparsematrix_amd import _lib
    rp = np.array([0, 1], np.int32)
    for bad in (dict(merge_stage=2), dict(band_tall=5), dict(layout=42)):
        o = _lib.build_opts(**bad)
        assert lib.sm_create_from_csr_ex(1, 4, 1, rp.ctypes.data, ci.ctypes.data, va.ctypes.data, 0,
                                         C.byref(o), C.byref(h)) == 1, bad


def test_python_mirror_surface():
    import sparsematrix_amd as smd
    for name in ("CopyForm", "CopyTo", "AddMatMat", "NumRows", "NumCols", "Destroy",
                 "SelfTest", "__eq__", "spmv", "spmm", "from_csr"):
        assert hasattr(smd.SparseMatrix, name)
    assert smd.SblasNoTrans == 0 and smd.SblasTrans == 1


def test_header_and_python_mirror_agree():
    """The sm_algo values and the sm_info layout the Python mirror uses match the C
    header (a struct mismatch would let sm_get_info write past the ctypes buffer)."""
    import ctypes
    import re
    import subprocess
    import tempfile

    from sparsematrix_amd import _lib
    hdr = open(os.path.join(ROOT, "include", "sparsematrix.h")).read()
    for name, val in _lib.ALGOS.items():
        m = re.search(r"SM_ALGO_%s\s*=\s*(\d+)" % name.upper(), hdr)
        assert m and int(m.group(1)) == val, name
    structs = (("sm_info", _lib.SmInfo), ("sm_build_opts", _lib.SmBuildOpts))
    body = "".join('printf("%%zu\\n", sizeof(%s));' % c + "".join(
        'printf("%%zu\\n", offsetof(%s, %s));' % (c, f) for f, _ in py._fields_) for c, py in structs)
    src = '#include <stddef.h>\n#include <stdio.h>\n#include "sparsematrix.h"\nint main(void){%sreturn 0;}\n' % body
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        got = iter(map(int, subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()))
    for cname, py in structs:   # every field of the ctypes mirror at the header's offset
        assert ctypes.sizeof(py) == next(got), cname
        for f, _ in py._fields_:
            assert getattr(py, f).offset == next(got), (cname, f)
