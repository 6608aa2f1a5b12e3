#!/usr/bin/env python3
"""R-MAT (config 4) sliced-ELL timeline: builds R-MAT scale S (AUTO:
the codebook sliced ELL over relabeled columns) and runs a few SpMVs with the development
library (SM_LIB_PATH=build/dev/libsparsematrix_amd.so) and SM_SELL_TS=1, which prints
per length class of slices their count, mean duration and last end, and when 50/90/99/100 %
of the slices had ended.  Also prints the slices' padding (padded slots / real terms)."""
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
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    rp, ci, va = synth.rmat_device(scale, 16, seed=4)
    n = 1 << scale
    M = smd.SparseMatrix.from_csr(rp, ci, va, n, device=0)
    info = M.info()
    print({k: info[k] for k in ("sell_slices", "sell_codebook", "col_relabel", "max_row_nnz", "nnz")}, flush=True)
    lens = (rp[1:] - rp[:-1]).cpu().numpy().astype(np.int64)
    seg = np.concatenate([np.minimum(lens[lens > 0], 2048),
                          np.full(int(np.sum(lens[lens > 2048] // 2048)), 2048)])
    # the builder's slices: rows <= 2048 and 2048-term segments sorted by length, 64 per slice,
    # each padded to its longest row rounded up to 8 (sell.cpp)
    seg = np.sort(seg)[::-1]
    k = (seg.size + 63) // 64
    pad = np.zeros(k * 64, np.int64)
    pad[:seg.size] = seg
    slice_max = pad.reshape(k, 64).max(axis=1)
    padded = int(np.sum((slice_max + 7) // 8 * 8) * 64)
    print(f"units {seg.size}, slices {k}, padded slots {padded}, real terms {int(seg.sum())}, "
          f"padding x{padded / max(1, seg.sum()):.3f}", flush=True)
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.rand(n, generator=g, device="cuda") * 2 - 1
    y = torch.rand(n, generator=g, device="cuda") * 2 - 1
    for _ in range(int(os.environ.get("RMAT_PROF_REPS", "3"))):
        M.spmv(x, y, 1.0, 0.5)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
