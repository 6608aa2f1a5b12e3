#!/usr/bin/env python3
"""AUTO's layout on small square matrices (16 distinct uniform columns per row): the band
layout it builds (tiles = row blocks x slabs: 16 tiles at 16K rows) against the sorted sliced
ELL (layout = no_bands) and the parity kernel.  Median of 50 eager SpMVs with HIP events."""
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
    print(f"{'n':>8s} {'auto layout':>12s} {'tiles':>6s} {'auto us':>8s} {'sell us':>8s} {'parity us':>9s}")
    for n in (16384, 32768, 65536, 131072, 262144, 524288):
        rp, ci, va = synth.uniform_rows_device(n, n, 16, seed=n)
        A = sm.SparseMatrix.from_csr(rp, ci, va, n)
        S = sm.SparseMatrix.from_csr(rp, ci, va, n, opts=dict(layout="no_bands"))
        ia = A.info()
        x = torch.rand(n, device="cuda") * 2 - 1
        y = torch.rand(n, device="cuda") * 2 - 1
        res = []
        for M, algo in ((A, "auto"), (S, "auto"), (A, "parity")):
            for _ in range(5):
                M.spmv(x, y, 1.0, 0.5, algo=algo)
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
            for a, b in ev:
                a.record()
                M.spmv(x, y, 1.0, 0.5, algo=algo)
                b.record()
            torch.cuda.synchronize()
            res.append(float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3)
        tiles = ia["xband_blocks"] * ia["xband_slabs"] if ia["has_xband"] else 0
        print(f"{n:8d} {('xband' + str(ia['has_xband'])) if ia['has_xband'] else 'sell':>12s} {tiles:6d} "
              f"{res[0]:8.1f} {res[1]:8.1f} {res[2]:9.1f}", flush=True)


if __name__ == "__main__":
    main()
