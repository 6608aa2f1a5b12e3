"""CopyForm timing: host encoder vs the device scan at n x n
(default 16384^2, 1 % density, T = 255).  Whole constructor, plans included; the
device variant starts from an index already in HBM.

    python tools/encode_bench.py [--n 16384] [--density 0.01] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--density", type=float, default=0.01)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    import sparsematrix_amd as smd
    smd.load()
    n = args.n
    g = torch.Generator(device="cuda").manual_seed(1)
    keep = torch.rand((n, n), generator=g, device="cuda") < args.density
    ids = torch.randint(0, 255, (n, n), generator=g, device="cuda", dtype=torch.uint8)
    d_index = torch.where(keep, ids, torch.full_like(ids, 255)).contiguous()
    h_index = d_index.cpu().numpy()
    table = np.random.default_rng(0).uniform(-1, 1, 255).astype(np.float32)
    out = {"n": n, "density": args.density}
    for trans in (0, 1):
        th, td = [], []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            H = smd.SparseMatrix(h_index, n, n, n, table, 255, trans)
            th.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            D = smd.SparseMatrix.from_dense_index(d_index.view(-1), n, n, n, table, 255, trans)
            torch.cuda.synchronize()
            td.append(time.perf_counter() - t0)
        same = all(np.array_equal(a.view(np.uint32), b.view(np.uint32))
                   for a, b in zip(H.csr(), D.csr()))
        out[f"trans{trans}"] = {"host_s": round(min(th), 4), "device_s": round(min(td), 4),
                                "nnz": H.info()["nnz"], "csr_identical": same}
        del H, D
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
