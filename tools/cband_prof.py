#!/usr/bin/env python3
"""Per-phase cycles of the cband SpMV on config 2 (development build:
SM_LIB_PATH=build/dev/libsparsematrix_amd.so SM_BAND2_PROF=1 -- dma3's cycles per band of
every phase, applying waves and loader -- or SM_BAND2_PROF=2 -- the per-tile timeline; add
SM_B2_TS_DUMP=1 for every tile's line).
Extra arguments: build options as key=value (e.g. band_slabs=2)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import sparsematrix_amd as smd
    from sparsematrix_amd import synth
    smd.load()
    opts = {k: int(v) for k, v in (a.split("=") for a in sys.argv[1:])}
    n = 1 << 20
    rp, ci, va = synth.uniform_rows_device(n, n, 16, seed=1, device="cuda")
    M = smd.SparseMatrix.from_csr(rp, ci, va, n, device=0, opts=opts or None)
    print({k: M.info()[k] for k in ("has_xband", "xband_slabs", "xband_block_rows")}, flush=True)
    x = torch.rand(n, device="cuda") * 2 - 1
    y = torch.rand(n, device="cuda") * 2 - 1
    for _ in range(4):
        M.spmv(x, y, 1.0, 0.5)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
