"""Synthetic inputs for the BASELINE configs, generated on the device with torch.

* ``uniform_rows_device`` -- config 2/3/5: every row holds exactly ``per_row``
  distinct, sorted, uniformly random columns.
* ``rmat_device`` -- config 4: Graph500-style R-MAT (a, b, c, d), directed,
  self-loops dropped, duplicates merged, vertex labels randomly permuted.
* ``banded_device`` -- a locality-friendly matrix (columns near the diagonal).

Values are drawn from one fixed 255-entry codebook, uniform[-1, 1) with seed
0x5EED, so small instances are also expressible in the
reference's codebook format.  torch is used here only as device memory and
RNG plumbing.
"""
from __future__ import annotations

import numpy as np

TABLE_SEED = 0x5EED


def codebook() -> np.ndarray:
    return np.random.default_rng(TABLE_SEED).uniform(-1.0, 1.0, 255).astype(np.float32)


def _values(torch, nnz: int, gen, device):
    table = torch.from_numpy(codebook()).to(device)
    ids = torch.randint(0, 255, (nnz,), generator=gen, device=device)
    return table[ids].contiguous()


def uniform_rows_device(n_rows: int, n_cols: int, per_row: int, seed: int, device="cuda"):
    """CSR (row_ptr int32, col_idx int32, val float32) torch tensors on `device`."""
    import torch
    assert per_row <= n_cols
    gen = torch.Generator(device=device).manual_seed(seed)
    cols = torch.randint(0, n_cols, (n_rows, per_row), generator=gen, device=device,
                         dtype=torch.int64)
    cols, _ = torch.sort(cols, dim=1)
    for _ in range(64):   # resample duplicates until every row is distinct
        dup = torch.zeros_like(cols, dtype=torch.bool)
        dup[:, 1:] = cols[:, 1:] == cols[:, :-1]
        nd = int(dup.sum())
        if nd == 0:
            break
        cols[dup] = torch.randint(0, n_cols, (nd,), generator=gen, device=device,
                                  dtype=torch.int64)
        cols, _ = torch.sort(cols, dim=1)
    else:
        raise RuntimeError("could not make rows distinct")
    col_idx = cols.reshape(-1).to(torch.int32).contiguous()
    row_ptr = (torch.arange(n_rows + 1, device=device, dtype=torch.int64) * per_row).to(torch.int32)
    val = _values(torch, n_rows * per_row, gen, device)
    return row_ptr, col_idx, val


def rmat_device(scale: int, edgefactor: int = 16, a: float = 0.57, b: float = 0.19,
                c: float = 0.19, seed: int = 4, permute: bool = True, device="cuda"):
    """Graph500 R-MAT edge list -> CSR of the directed adjacency (row = source)."""
    import torch
    n = 1 << scale
    m = edgefactor * n
    gen = torch.Generator(device=device).manual_seed(seed)
    src = torch.zeros(m, dtype=torch.int64, device=device)
    dst = torch.zeros(m, dtype=torch.int64, device=device)
    ab, abc = a + b, a + b + c
    for level in range(scale):
        r = torch.rand(m, generator=gen, device=device)
        src |= (r >= ab).to(torch.int64) << level
        dst |= (((r >= a) & (r < ab)) | (r >= abc)).to(torch.int64) << level
        del r
    if permute:
        perm = torch.randperm(n, generator=gen, device=device)
        src = perm[src]
        dst = perm[dst]
    keep = src != dst
    key = torch.unique(src[keep] * n + dst[keep])   # sorted, duplicates merged
    del src, dst, keep
    rows = key // n
    col_idx = (key % n).to(torch.int32).contiguous()
    counts = torch.bincount(rows, minlength=n)
    row_ptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
    row_ptr[1:] = torch.cumsum(counts, 0)
    val = _values(torch, int(col_idx.numel()), gen, device)
    return row_ptr.to(torch.int32), col_idx, val


def banded_device(n_rows: int, per_row: int, band: int, seed: int, device="cuda"):
    """Rows with `per_row` distinct columns within +-band of the diagonal."""
    import torch
    gen = torch.Generator(device=device).manual_seed(seed)
    span = 2 * band + 1
    assert per_row <= span
    off = torch.rand((n_rows, span), generator=gen, device=device).argsort(dim=1)[:, :per_row]
    off, _ = torch.sort(off, dim=1)
    r = torch.arange(n_rows, device=device).unsqueeze(1)
    cols = (r - band + off).clamp_(0, n_rows - 1)
    cols, _ = torch.sort(cols, dim=1)
    # clamping can collide at the edges: keep it simple, dedupe by nudging
    cols[:, 1:] = torch.maximum(cols[:, 1:], cols[:, :-1] + 1)
    cols.clamp_(max=n_rows - 1)
    col_idx = cols.reshape(-1).to(torch.int32).contiguous()
    row_ptr = (torch.arange(n_rows + 1, device=device, dtype=torch.int64) * per_row).to(torch.int32)
    return row_ptr, col_idx, _values(torch, n_rows * per_row, gen, device)
