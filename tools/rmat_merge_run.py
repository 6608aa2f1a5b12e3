#!/usr/bin/env python3
"""SM_ALGO_MERGE on BASELINE config 4 (R-MAT scale 24, edgefactor 16, seed 4, as bench.py builds
it): both plans -- the CSR arrays (spmv_merge_kernel<false>) and the column-sorted staging copy
(sm_build_opts.merge_stage, spmv_merge_kernel<true>) -- K SpMVs each after warmup, HIP-event
median per SpMV (and AUTO's codebook sliced ELL beside them, RMAT_AUTO=1).  Under rocprofv3 --pmc this is the command tools/pmc.sh profiles
(PMC_CMD) for profiles/traffic_rmat24_merge*.json."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import sparsematrix_amd as smd
    from sparsematrix_amd import synth
    smd.load()
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    rp, ci, va = synth.rmat_device(24, 16, seed=4)
    n = 1 << 24
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y = torch.rand(n, device="cuda", generator=g) * 2 - 1
    out = {}
    if os.environ.get("RMAT_AUTO", "1") == "1":   # the AUTO layout (codebook sliced ELL) beside it
        M = smd.SparseMatrix.from_csr(rp, ci, va, n)
        for _ in range(3):
            M.spmv(x, y, 1.0, 0.5)
        torch.cuda.synchronize()
        ts = []
        for _ in range(steps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            M.spmv(x, y, 1.0, 0.5)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        out["auto_ms"] = round(float(np.median(ts)), 4)
        del M
        torch.cuda.empty_cache()
    for stage in (0, 1):
        M = smd.SparseMatrix.from_csr(rp, ci, va, n, opts={"merge_stage": stage})
        for _ in range(3):
            M.spmv(x, y, 1.0, 0.5, algo="merge")
        torch.cuda.synchronize()
        ts = []
        for _ in range(steps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            M.spmv(x, y, 1.0, 0.5, algo="merge")
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        out["staged_ms" if stage else "ms"] = round(float(np.median(ts)), 4)
        del M
        torch.cuda.empty_cache()
    print(json.dumps({"rmat24_merge": out}), flush=True)


if __name__ == "__main__":
    main()
