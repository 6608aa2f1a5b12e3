#!/usr/bin/env python3
"""Config 4 (R-MAT scale 24) on gathered chunk bands (gcb) against AUTO's
codebook sliced ELL -- VERDICT r4 item 2.

gcb keeps a tile's row sums in LDS and walks the tile's terms in (column, row) order in
bands of < 2^18 columns, so the tile's gathers of one x line come close together.  R-MAT's
hub columns get the same treatment as AUTO's sliced ELL: the columns are relabeled by
descending degree (a dense hot prefix of x that stays in L2), each row's terms re-sorted by
the new labels, and x is permuted per SpMV (timed separately: the same scatter AUTO runs).
Timing: HIP events around each SpMV, median of 20 eager launches (as tools/rmat_ab.py).

Usage: rmat_gcb_ab.py [scale] [slabs ...]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import sparsematrix_amd as smd
    from sparsematrix_amd import synth
    smd.load()
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    slab_list = [int(s) for s in sys.argv[2:]] or [0]
    dev = torch.device("cuda:0")
    rp, ci, va = synth.rmat_device(scale, 16, seed=4)
    n = 1 << scale
    nnz = int(ci.numel())
    g = torch.Generator(device=dev).manual_seed(4)
    x = torch.rand(n, generator=g, device=dev) * 2 - 1
    y = torch.rand(n, generator=g, device=dev) * 2 - 1
    alg = 8 * nnz + 4 * (n + 1) + 4 * n + 8 * n

    def timed(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in ev]))

    # AUTO (codebook sliced ELL on relabeled columns)
    t0 = time.perf_counter()
    M = smd.SparseMatrix.from_csr(rp, ci, va, n, device=0)
    torch.cuda.synchronize()
    b_auto = time.perf_counter() - t0
    ms = timed(lambda: M.spmv(x, y, 1.0, 0.5))
    info = M.info()
    print(f"AUTO        {ms:8.4f} ms  {alg / ms / 1e6:7.1f} GB/s  build {b_auto:5.1f} s  has_xband={info['has_xband']} "
          f"sell_slices={info['sell_slices']} col_relabel={info['col_relabel']}", flush=True)
    del M
    torch.cuda.empty_cache()

    # relabel by descending degree, rows re-sorted by the new labels
    deg = torch.bincount(ci.long(), minlength=n)
    order = torch.argsort(deg, descending=True, stable=True)          # new -> old
    rank = torch.empty_like(order)
    rank[order] = torch.arange(n, device=dev)                          # old -> new
    row = torch.repeat_interleave(torch.arange(n, device=dev), (rp[1:] - rp[:-1]).long())
    key = row * n + rank[ci.long()]
    perm = torch.argsort(key)
    ci2 = (key[perm] % n).to(torch.int32)
    va2 = va[perm].contiguous()
    del key, perm, row
    xp = torch.empty_like(x)
    order32 = order.to(torch.int64)
    ms_perm = timed(lambda: xp.copy_(x[order32]))
    print(f"x permutation (torch gather) {ms_perm:8.4f} ms", flush=True)
    lens = (rp[1:] - rp[:-1]).long()
    tile_terms = torch.zeros((n + 32767) // 32768, dtype=torch.long, device=dev)
    tile_terms.index_add_(0, torch.arange(n, device=dev) // 32768, lens)
    print(f"terms per 32K-row tile: max {int(tile_terms.max())} mean {float(tile_terms.float().mean()):.0f} "
          f"(max/mean {float(tile_terms.max()) / float(tile_terms.float().mean()):.1f}); the longest tile is one "
          f"CU's serial work", flush=True)
    variants = [(s, False) for s in slab_list] + ([] if os.environ.get("RMAT_GCB_NO_SHUFFLE") else [(slab_list[0], True)])
    for slabs, shuffle in variants:
        rpv, civ, vav = rp, ci2, va2
        if shuffle:   # rows in random order: every tile gets ~ the mean (y gathered / scattered per SpMV)
            g2 = torch.Generator(device=dev).manual_seed(11)
            rperm = torch.randperm(n, generator=g2, device=dev)
            l2 = lens[rperm]
            rpv = torch.zeros(n + 1, dtype=torch.long, device=dev)
            rpv[1:] = torch.cumsum(l2, 0)
            rowv = torch.repeat_interleave(torch.arange(n, device=dev), l2)
            src = rp.long()[rperm][rowv] + (torch.arange(nnz, device=dev) - rpv[rowv])
            civ, vav = ci2[src].contiguous(), va2[src].contiguous()
            rpv = rpv.to(torch.int32)
            del rowv, src
            tt = torch.zeros_like(tile_terms)
            tt.index_add_(0, torch.arange(n, device=dev) // 32768, l2)
            print(f"shuffled rows: terms per tile max {int(tt.max())}", flush=True)
            yv = torch.empty_like(y)
            ms_y = timed(lambda: (yv.copy_(y[rperm]), y.index_copy_(0, rperm, yv)))
            print(f"y gather + scatter (torch) {ms_y:8.4f} ms", flush=True)

        t0 = time.perf_counter()
        try:
            M = smd.SparseMatrix.from_csr(rpv, civ, vav, n, device=0,
                                          opts={"layout": "gcb", "band_slabs": slabs, "relabel": 0})
        except Exception as e:  # noqa: BLE001 - report and go on
            print(f"gcb slabs={slabs} shuffle={shuffle}: build failed: {e}", flush=True)
            continue
        torch.cuda.synchronize()
        b = time.perf_counter() - t0
        info = M.info()
        xp.copy_(x[order32])
        ms = timed(lambda: M.spmv(xp, y, 1.0, 0.5))
        print(f"gcb {'shuffled ' if shuffle else ''}slabs={slabs:2d} {ms:8.4f} ms (+ permutation) {alg / (ms + ms_perm) / 1e6:7.1f} GB/s  build {b:5.1f} s "
              f"has_xband={info['has_xband']} blocks={info['xband_blocks']} slabs={info['xband_slabs']} "
              f"bands={info['xband_bands']} block_rows={info['xband_block_rows']}", flush=True)
        del M
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
