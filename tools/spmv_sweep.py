#!/usr/bin/env python3
"""Interleaved A/B timing of SpMV variants on one GPU, one process.

Variants: stream kernel at each tile size (SM_TILE_NNZ, read at matrix
creation), the CSR-vector kernel and the parity kernel.  Replicas rotate so
the working set exceeds the 256 MiB Infinity Cache.  Prints one line per
variant: median / min kernel time and GB/s on the algorithmic bytes.

  python tools/spmv_sweep.py [--workload uniform|rmat|banded] [--rows N] ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="uniform")
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--per-row", type=int, default=16)
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--replicas", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tiles", default="1024,2048,4096,8192")
    ap.add_argument("--algos", default="xband,vector,parity")
    ap.add_argument("--json", default="")
    ap.add_argument("--ablate", default="", help="xband ablation modes (dev), e.g. 1,2,4")
    ap.add_argument("--opts", default="{}", help='sm_build_opts for the --algos matrices, JSON, '
                    'e.g. \'{"merge_stage": 1}\'')
    args = ap.parse_args()

    import torch

    import sparsematrix_amd as smd
    from sparsematrix_amd import synth

    smd.load()
    dev = torch.device("cuda", 0)
    data = []
    for k in range(args.replicas):
        if args.workload == "uniform":
            rp, ci, va = synth.uniform_rows_device(args.rows, args.rows, args.per_row, seed=2 + k)
            ncols = args.rows
        elif args.workload == "rmat":
            rp, ci, va = synth.rmat_device(args.scale, 16, seed=4 + k)
            ncols = 1 << args.scale
        elif args.workload == "banded":
            rp, ci, va = synth.banded_device(args.rows, args.per_row, 64, seed=2 + k)
            ncols = args.rows
        else:
            raise SystemExit("unknown workload")
        g = torch.Generator(device=dev).manual_seed(100 + k)
        x = torch.rand(ncols, generator=g, device=dev) * 2 - 1
        y = torch.rand(rp.numel() - 1, generator=g, device=dev) * 2 - 1
        data.append((rp, ci, va, ncols, x, y))
    n_rows = data[0][0].numel() - 1
    nnz = int(data[0][1].numel())
    alg = 8 * nnz + 4 * (n_rows + 1) + 4 * data[0][3] + 8 * n_rows

    variants = []
    for tsz in [int(t) for t in args.tiles.split(",") if t]:
        os.environ["SM_TILE_NNZ"] = str(tsz)
        mats = [smd.SparseMatrix.from_csr(rp, ci, va, nc) for rp, ci, va, nc, _, _ in data]
        variants.append((f"stream/tile{tsz}", "stream", mats))
    os.environ.pop("SM_TILE_NNZ", None)
    xmats = None
    for kind, name in (("blocked", "xband"), ("exact", "exact")):
        if name not in args.algos.split(","):
            continue
        os.environ["SM_XBAND"] = "1"
        os.environ["SM_XBAND_KIND"] = kind
        mats = [smd.SparseMatrix.from_csr(rp, ci, va, nc) for rp, ci, va, nc, _, _ in data]
        os.environ.pop("SM_XBAND")
        os.environ.pop("SM_XBAND_KIND")
        print(f"{name} layout:", {k: mats[0].info()[k] for k in (
            "has_xband", "xband_blocks", "xband_bands", "xband_slabs", "xband_block_rows")})
        variants.append((name, "xband", mats))
        xmats = xmats or mats
    for a in [int(v) for v in args.ablate.split(",") if v]:
        variants.append((f"xband/ablate{a}", ("xband", a), xmats))
    os.environ["SM_XBAND"] = "0"
    base_mats = [smd.SparseMatrix.from_csr(rp, ci, va, nc, opts=json.loads(args.opts))
                 for rp, ci, va, nc, _, _ in data]
    os.environ.pop("SM_XBAND")
    for a in [a for a in args.algos.split(",") if a and a not in ("xband", "exact")]:
        variants.append((a, a, base_mats))
    info = base_mats[0].info()

    times = {name: [] for name, _, _ in variants}
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.reps)]
    for rnd in range(args.rounds):
        for name, algo, mats in variants:
            os.environ.pop("SM_XBAND_ABLATE", None)
            if isinstance(algo, tuple):
                algo, abl = algo
                os.environ["SM_XBAND_ABLATE"] = str(abl)
            for i in range(3):
                d = data[i % len(data)]
                mats[i % len(mats)].spmv(d[4], d[5], 1.0, 0.5, algo=algo)
            for i, (a, b) in enumerate(ev):
                d = data[i % len(data)]
                a.record()
                mats[i % len(mats)].spmv(d[4], d[5], 1.0, 0.5, algo=algo)
                b.record()
            torch.cuda.synchronize()
            times[name] += [a.elapsed_time(b) for a, b in ev]
    out = {"workload": args.workload, "n_rows": n_rows, "nnz": nnz, "alg_bytes": alg,
           "max_row_nnz": info["max_row_nnz"], "n_long_rows": info["n_long_rows"], "variants": {}}
    print(f"workload={args.workload} rows={n_rows} nnz={nnz} alg_bytes={alg} "
          f"max_row={info['max_row_nnz']} long_rows={info['n_long_rows']}")
    for name, _, _ in variants:
        t = np.array(times[name])
        med, mn = float(np.median(t)), float(t.min())
        out["variants"][name] = {"median_ms": med, "min_ms": mn, "gbs_median": alg / med / 1e6}
        print(f"  {name:18s} median {med * 1e3:8.1f} us  min {mn * 1e3:8.1f} us  "
              f"{alg / med / 1e6:8.1f} GB/s  ({alg / med / 1e6 / 8000:.3f} of 8 TB/s)")
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
