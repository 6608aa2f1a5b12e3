"""Development: per-band phase timing of the band kernel from in-kernel s_memtime
stamps (SM_XBAND_ABLATE=32: full kernel; 37: x staging only).  Tile 0, 16 waves.
Prints median cycles per phase: [store slice] [issue loads + apply] [barrier]."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import sparsematrix_amd as smd
    from sparsematrix_amd import synth

    smd.load()
    rp, ci, va = synth.uniform_rows_device(1 << 20, 1 << 20, 16, seed=2)
    os.environ["SM_XBAND"] = "1"
    os.environ["SM_XBAND_KIND"] = sys.argv[1] if len(sys.argv) > 1 else "blocked"
    M = smd.SparseMatrix.from_csr(rp, ci, va, 1 << 20)
    dev = torch.device("cuda", 0)
    x = torch.rand(1 << 20, device=dev)
    for abl in (32,):
        os.environ["SM_XBAND_ABLATE"] = str(abl)
        for _ in range(3):
            y = torch.zeros(1 << 20, device=dev)
            M.spmv(x, y, 1.0, 1.0, algo="xband")
        torch.cuda.synchronize()
        t = y[:3072].cpu().numpy().view(np.uint32).astype(np.int64).reshape(16, 32, 6)
        t0 = t[:, :, 0]
        names = ["store", "issue", "entries", "apply", "barrier"]
        ph = [t[:, :, k + 1] - t[:, :, k] for k in range(5)]
        ph.append(np.diff(np.concatenate([t0, t0[:, -1:]], 1), axis=1))
        ph = np.stack(ph, -1)
        med = np.median(ph[:, 1:31], axis=(0, 1))
        print(f"ABL {abl}: cycles/band " + "  ".join(f"{n} {m:.0f}" for n, m in zip(names, med))
              + f"  total {med[5]:.0f}")
        for k, n in enumerate(names + ["total"]):
            print(f"   per-wave {n:8s}", np.median(ph[:, 1:31, k], axis=1).astype(int).tolist())
    os.environ.pop("SM_XBAND_ABLATE")


if __name__ == "__main__":
    main()
