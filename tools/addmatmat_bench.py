"""AddMatMat (m right-hand rows, row-major A m x k and C m x n) on the device:
the in-place one-thread-per-output kernel (algo="parity") vs the row-panel path
(algo="auto": transposes + spmm_rowpanel2 + transpose back).  Config-2 matrix.

    python tools/addmatmat_bench.py [--m 32] [--reps 10]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--m", default="8,32")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch

    import sparsematrix_amd as smd
    from sparsematrix_amd import synth
    smd.load()
    dev = torch.device("cuda", 0)
    R = args.rows
    rp, ci, va = synth.uniform_rows_device(R, R, 16, seed=2, device=dev)
    M = smd.SparseMatrix.from_csr(rp, ci, va, R)
    for m in (int(v) for v in args.m.split(",")):
        g = torch.Generator(device=dev).manual_seed(3)
        A = torch.rand((m, R), generator=g, device=dev) * 2 - 1
        C0 = torch.rand((m, R), generator=g, device=dev) * 2 - 1
        res = {}
        for algo in ("parity", "auto"):
            C = C0.clone()
            M.AddMatMat(A, m, R, C, R, 1.0, 0.5, algo=algo)
            torch.cuda.synchronize()
            out = C.cpu().numpy().view(np.uint32)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.reps)]
            for a, b in ev:
                a.record()
                M.AddMatMat(A, m, R, C, R, 1.0, 0.5, algo=algo)
                b.record()
            torch.cuda.synchronize()
            res[algo] = (float(np.median([a.elapsed_time(b) for a, b in ev])), out)
        print(json.dumps({"m": m, "parity_ms": round(res["parity"][0], 3),
                          "auto_ms": round(res["auto"][0], 3),
                          "bit_identical": bool(np.array_equal(res["parity"][1], res["auto"][1]))}),
              flush=True)


if __name__ == "__main__":
    main()
