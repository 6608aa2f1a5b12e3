"""Host logic of the column-band layout builder (sparsematrix_amd/csrc/xband.cpp),
no GPU: tests/native/xband_asan.cpp is compiled with AddressSanitizer and run.
It rebuilds every row from the layout (both the exact and the blocked bit layout)
and checks order, ranks, register capacity and the dummy encoding."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_xband_builder_under_asan(tmp_path):
    exe = tmp_path / "xband_asan"
    src = [os.path.join(ROOT, "tests", "native", "xband_asan.cpp"),
           os.path.join(ROOT, "sparsematrix_amd", "csrc", "xband.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "sparsematrix_amd", "csrc"),
                    *src, "-o", str(exe), "-pthread"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "xband_asan: ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_band2_builder_under_asan(tmp_path):
    """Balanced-band builder (band2.cpp): every term once, per row in ascending column
    order, segments on consecutive lanes with their ranks, band windows respected."""
    exe = tmp_path / "band2_asan"
    src = [os.path.join(ROOT, "tests", "native", "band2_asan.cpp"),
           os.path.join(ROOT, "sparsematrix_amd", "csrc", "band2.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "sparsematrix_amd", "csrc"),
                    *src, "-o", str(exe), "-pthread"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "band2_asan: ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_sell_builder_under_asan(tmp_path):
    """Sorted sliced-ELL builder (sell.cpp): every short row in exactly one lane with its
    terms in stored order, long rows in consecutive segments, slices sorted and padded."""
    exe = tmp_path / "sell_asan"
    src = [os.path.join(ROOT, "tests", "native", "sell_asan.cpp"),
           os.path.join(ROOT, "sparsematrix_amd", "csrc", "sell.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "sparsematrix_amd", "csrc"),
                    *src, "-o", str(exe), "-pthread"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sell_asan: ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_ccsell_builder_under_asan(tmp_path):
    """Column-chunked sliced-ELL builder (ccsell.cpp): walking chunks in order, every row's
    terms once in ascending column order, one first-flagged unit per row, sorted slices."""
    exe = tmp_path / "ccsell_asan"
    src = [os.path.join(ROOT, "tests", "native", "ccsell_asan.cpp"),
           os.path.join(ROOT, "sparsematrix_amd", "csrc", "ccsell.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "sparsematrix_amd", "csrc"),
                    *src, "-o", str(exe), "-pthread"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ccsell_asan: ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_encode_csr_ref_under_asan(tmp_path):
    """CSR -> reference-stream converter (encode.cpp encode_csr_ref, behind
    sm_build_ref_stream): the dense encoder's CSR converted back gives its stream, panels
    and table exactly (the dense encoder is pinned to the compiled reference by the golden
    fixtures); a derived codebook decodes to the same values; bad inputs decline."""
    exe = tmp_path / "encode_csr_asan"
    src = [os.path.join(ROOT, "tests", "native", "encode_csr_asan.cpp"),
           os.path.join(ROOT, "sparsematrix_amd", "csrc", "encode.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "sparsematrix_amd", "csrc"),
                    *src, "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "encode_csr_asan: ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_sweep_builder_under_asan(tmp_path):
    """Column-swept row-block builder (sweep.cpp): each block's chunks, walked in order,
    give every row's terms once in ascending column order with their ids; segments are
    contiguous with continuation bits; padding is dummy; unsorted rows decline."""
    exe = tmp_path / "sweep_asan"
    src = [os.path.join(ROOT, "tests", "native", "sweep_asan.cpp"),
           os.path.join(ROOT, "sparsematrix_amd", "csrc", "sweep.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "sparsematrix_amd", "csrc"),
                    *src, "-o", str(exe), "-pthread"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sweep_asan: ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_gcb_builder_under_asan(tmp_path):
    """Gathered-chunk-band builder (gcb.cpp), decoded as the kernel decodes it: every term
    once, rows in ascending column order, segments on consecutive lanes of one chunk, one
    chunk per row per band, windows and slabs respected, padding as dummies."""
    exe = tmp_path / "gcb_asan"
    src = [os.path.join(ROOT, "tests", "native", "gcb_asan.cpp"),
           os.path.join(ROOT, "sparsematrix_amd", "csrc", "gcb.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "sparsematrix_amd", "csrc"),
                    *src, "-o", str(exe), "-pthread"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gcb_asan: ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_merge_plan_under_asan(tmp_path):
    """Merge path's plan (merge.cpp): slice corners against a sequential walk of the merge,
    and the column-sorted staging stream (a per-slice permutation, ascending columns with ties
    in CSR order, codebook ids back to the values' bits; declined past 255 values / 2^24 cols)."""
    exe = tmp_path / "merge_asan"
    src = [os.path.join(ROOT, "tests", "native", "merge_asan.cpp"),
           os.path.join(ROOT, "sparsematrix_amd", "csrc", "merge.cpp"),
           os.path.join(ROOT, "sparsematrix_amd", "csrc", "band2.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "sparsematrix_amd", "csrc"),
                    *src, "-o", str(exe), "-pthread"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "merge_asan: ok" in r.stdout
