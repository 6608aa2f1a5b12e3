"""R-MAT scale 24 column-degree concentration (after relabeling by degree) and the share
of terms in rows longer than 2048 (development probe for the sell kernel)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparsematrix_amd import synth  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
rp, ci, va = synth.rmat_device(scale, 16, seed=4)
n = 1 << scale
deg = torch.bincount(ci.long(), minlength=n)
d = torch.sort(deg, descending=True).values.double()
cs = d.cumsum(0) / d.sum()
for k in (4096, 8192, 16384, 32768, 65536, 1 << 17, 1 << 18, 1 << 20):
    print(f"top {k:8d} columns hold {cs[k - 1].item():.3f} of the terms")
lens = (rp[1:] - rp[:-1]).double()
print("nnz", ci.numel(), "share in rows > 2048 terms",
      round((lens * (lens > 2048)).sum().item() / ci.numel(), 3),
      "empty rows", round((lens == 0).double().mean().item(), 3))
