#!/usr/bin/env python3
"""Development check of a band2 / cband slab hand-off build (SM_LIB_PATH = a -DSM_DEV build):
config 2 and two smaller shapes, several launches and graph replays, every result bit for bit
against the slab-order restatement (tests/gpu_util.slab_order_for) for the geometry and hand-off
form the matrix reports."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import torch

    import sparsematrix_amd as smd
    from sparsematrix_amd import synth
    from gpu_util import bits, slab_order_for, uniform_csr
    smd.load()
    shapes = [("config2", None), ("300000x400000", (300000, 400000, 16, 31)), ("70000x900000", (70000, 900000, 12, 5))]
    for name, sh in shapes:
        if sh is None:
            n = 1 << 20
            rp, ci, va = synth.uniform_rows_device(n, n, 16, seed=2)
            rp, ci, va = rp.cpu().numpy(), ci.cpu().numpy(), va.cpu().numpy()
            n_cols = n
        else:
            rp, ci, va = uniform_csr(sh[0], sh[1], sh[2], seed=sh[3])
            n_cols = sh[1]
        M = smd.SparseMatrix.from_csr(rp, ci, va, n_cols)
        info = M.info()
        g = torch.Generator(device="cuda").manual_seed(3)
        x = torch.rand(n_cols, device="cuda", generator=g) * 2 - 1
        y0 = torch.rand(rp.size - 1, device="cuda", generator=g) * 2 - 1
        xh, y0h = x.cpu().numpy(), y0.cpu().numpy()
        for alpha, beta in ((1.0, 0.5), (1.3, 1.0), (0.7, 0.0)):
            want = bits(slab_order_for(info, rp, ci, va, xh, y0h, alpha, beta))
            for rep in range(3):
                y = y0.clone()
                M.spmv(x, y, alpha, beta)
                torch.cuda.synchronize()
                ok = np.array_equal(bits(y.cpu().numpy()), want)
                if not ok:
                    print(name, "MISMATCH", alpha, beta, rep, {k: info[k] for k in (
                        "has_xband", "xband_slabs", "xband_slab_cols", "xband_beta_last")})
                    sys.exit(3)
        # graph replays of 5 SpMVs on one y: compare with 5 eager ones
        y = y0.clone()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(5):
                M.spmv(x, y, 1.0, 0.5)
        ye = y0.clone()
        for _ in range(5):
            M.spmv(x, ye, 1.0, 0.5)
        for _ in range(3):
            y.copy_(y0)
            graph.replay()
            torch.cuda.synchronize()
            assert torch.equal(y.view(torch.int32), ye.view(torch.int32)), name
        print(name, "ok", {k: info[k] for k in ("has_xband", "xband_slabs", "xband_slab_cols",
                                                 "xband_beta_last")}, flush=True)


if __name__ == "__main__":
    main()
