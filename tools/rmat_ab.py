#!/usr/bin/env python3
"""Config 4 (R-MAT scale 24) layout A/B: the same graph built with several
sm_build_opts variants, each timed as bench.py times it (HIP events around each
SpMV, median of 20 eager launches).  Usage: rmat_ab.py [scale] [variant ...] where a
variant is a Python dict literal of build options, e.g. "{'hot_cols': -1}"."""
import ast
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import sparsematrix_amd as smd
    from sparsematrix_amd import synth
    smd.load()
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    variants = [ast.literal_eval(v) for v in sys.argv[2:]] or [{}, {"hot_cols": -1}]
    dev = torch.device("cuda:0")
    rp, ci, va = synth.rmat_device(scale, 16, seed=4)
    n = 1 << scale
    g = torch.Generator(device=dev).manual_seed(4)
    x = torch.rand(n, generator=g, device=dev) * 2 - 1
    y = torch.rand(n, generator=g, device=dev) * 2 - 1
    nnz = int(ci.numel())
    alg = 8 * nnz + 4 * (n + 1) + 4 * n + 8 * n
    for opts in variants:
        t0 = time.perf_counter()
        M = smd.SparseMatrix.from_csr(rp, ci, va, n, device=0, opts=opts)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        info = M.info()
        for _ in range(3):
            M.spmv(x, y, 1.0, 0.5)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(20)]
        for a, b in ev:
            a.record()
            M.spmv(x, y, 1.0, 0.5)
            b.record()
        torch.cuda.synchronize()
        ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
        keys = ("has_xband", "sell_slices", "sell_codebook", "col_relabel", "hot_cols",
                "ccsell_chunks", "n_long_rows")
        print(f"{str(opts):36s} {ms:8.4f} ms  {alg / ms / 1e6:7.1f} GB/s  build {t1 - t0:5.1f} s  "
              + " ".join(f"{k}={info.get(k)}" for k in keys), flush=True)
        del M
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
