#!/usr/bin/env python3
"""Per-phase cycles of the native AddMatMat kernel (development build, SM_NAT_PROF=1,
SM_LIB_PATH=build/dev/libsparsematrix_amd.so): one warm launch, then one profiled launch
per case; the kernel prints kcycles per workgroup for each phase to stderr."""
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
    for name, n, dens in (("config1", 1024, 0.01), ("16k 0.1%", 16384, 0.001),
                          ("4096 25%", 4096, 0.25)):
        rng = np.random.default_rng(n)
        dm = np.where(rng.random((n, n)) < dens, rng.integers(0, 255, (n, n)), 255).astype(np.uint8)
        M = sm.SparseMatrix(dm, n, n, n, table, 255, sm.SblasTrans)
        for m in (1, 32):
            A = torch.rand(m * n, device="cuda") * 2 - 1
            C = torch.rand(m * n, device="cuda") * 2 - 1
            os.environ.pop("SM_NAT_PROF", None)
            M.AddMatMat(A, m, n, C, n, 1.0, 1.0, algo="native")
            torch.cuda.synchronize()
            print(f"{name} m={m}", file=sys.stderr, flush=True)
            os.environ["SM_NAT_PROF"] = "1"
            M.AddMatMat(A, m, n, C, n, 1.0, 1.0, algo="native")
            torch.cuda.synchronize()
            os.environ.pop("SM_NAT_PROF", None)


if __name__ == "__main__":
    main()
