import os, sys, time
sys.path.insert(0, "/root/repo")
import numpy as np, torch
import sparsematrix_amd as smd
from sparsematrix_amd import synth
smd.load()
dev = torch.device("cuda", 0)
scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
rp, ci, va = synth.rmat_device(scale, 16, seed=4)
n = 1 << scale
nnz = ci.numel()
deg = torch.bincount(ci.long(), minlength=n)
order = torch.argsort(deg, descending=True, stable=True)      # new label -> old column
rank = torch.empty_like(order); rank[order] = torch.arange(n, device=dev)  # old -> new
ci2 = rank[ci.long()].to(torch.int32)
sd = deg[order].double().cumsum(0) / nnz
for k in (1 << 14, 1 << 16, 1 << 18, 1 << 19, 1 << 20, 1 << 21):
    print(f"top {k:8d} cols ({k*4/2**20:6.2f} MiB) hold {sd[k-1].item():.3f} of terms")
os.environ["SM_XBAND"] = "0"
M1 = smd.SparseMatrix.from_csr(rp, ci, va, n)
M2 = smd.SparseMatrix.from_csr(rp, ci2, va, n)
x = torch.rand(n, device=dev) * 2 - 1
x2 = x[order]
y0 = torch.rand(n, device=dev)
def t(M, xx, algo="stream", reps=10):
    y = y0.clone()
    for _ in range(3): M.spmv(xx, y, 1.0, 0.5, algo=algo)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(); M.spmv(xx, y, 1.0, 0.5, algo=algo); b.record()
    torch.cuda.synchronize()
    return np.median([a.elapsed_time(b) for a, b in ev])
ya = y0.clone(); M1.spmv(x, ya, 1.0, 0.5, algo="stream")
yb = y0.clone(); M2.spmv(x2, yb, 1.0, 0.5, algo="stream")
torch.cuda.synchronize()
print("max |diff| orig vs relabeled:", (ya - yb).abs().max().item())
def perm_time(reps=10):
    for _ in range(3): xx = x[order]
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(); xx = torch.index_select(x, 0, order); b.record()
    torch.cuda.synchronize()
    return np.median([a.elapsed_time(b) for a, b in ev])
for algo in ("stream", "vector"):
    print(f"{algo}: original {t(M1, x, algo):.3f} ms   relabeled {t(M2, x2, algo):.3f} ms")
print(f"x permutation (index_select) {perm_time():.3f} ms")
