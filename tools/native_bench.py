#!/usr/bin/env python3
"""Device AddMatMat on the reference's own stream (SM_ALGO_NATIVE, native.hip) against
the CSR paths of the same matrix: config 1 (1024^2, 1 %), 16k^2 at 0.1 % (fillers
dominate the stream), and denser cases where the 2-byte stream beats 8-byte CSR.
Median of 50 launches with HIP events, m = 1 and m = 32; matrices built from the dense
uint8 index exactly as the reference's CopyForm (Trans).  Filters (for profiling runs):
NATIVE_CASES (substrings of the case names, comma-separated), NATIVE_M ("1,32"),
NATIVE_ALGOS ("native,auto,parity")."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import sparsematrix_amd as sm
    from sparsematrix_amd import synth
    sm.load()
    table = synth.codebook()
    cases = [("config1 1024^2 1%", 1024, 0.01), ("16384^2 0.1%", 16384, 0.001),
             ("4096^2 25%", 4096, 0.25), ("8192^2 5%", 8192, 0.05)]
    print(f"{'case':22s} {'m':>3s} {'entries':>10s} {'nnz':>10s} {'native us':>10s} "
          f"{'auto us':>9s} {'parity us':>10s}")
    sel = [c for c in os.environ.get("NATIVE_CASES", "").split(",") if c]
    if sel:
        cases = [c for c in cases if any(s in c[0] for s in sel)]
    ms = [int(v) for v in os.environ.get("NATIVE_M", "1,32").split(",")]
    algos = os.environ.get("NATIVE_ALGOS", "native,auto,parity").split(",")
    for name, n, dens in cases:
        rng = np.random.default_rng(n)
        dm = np.where(rng.random((n, n)) < dens, rng.integers(0, 255, (n, n)), 255).astype(np.uint8)
        M = sm.SparseMatrix(dm, n, n, n, table, 255, sm.SblasTrans)
        info = M.info()
        for m in ms:
            A = torch.rand(m * n, device="cuda") * 2 - 1
            C = torch.rand(m * n, device="cuda") * 2 - 1
            res = {"native": float("nan"), "auto": float("nan"), "parity": float("nan")}
            for algo in algos:
                for _ in range(5):
                    M.AddMatMat(A, m, n, C, n, 1.0, 1.0, algo=algo)
                torch.cuda.synchronize()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(50)]
                for a, b in ev:
                    a.record()
                    M.AddMatMat(A, m, n, C, n, 1.0, 1.0, algo=algo)
                    b.record()
                torch.cuda.synchronize()
                res[algo] = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3
            print(f"{name:22s} {m:3d} {info['n_entries']:10d} {info['nnz']:10d} "
                  f"{res['native']:10.1f} {res['auto']:9.1f} {res['parity']:10.1f}", flush=True)


if __name__ == "__main__":
    main()
