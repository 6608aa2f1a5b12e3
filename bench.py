#!/usr/bin/env python3
"""bench.py -- CSR SpMV effective HBM GB/s on MI355X (BASELINE.json metric).

Default (N=1): BASELINE config 2 -- B is 2^20 x 2^20 with exactly 16 distinct
uniformly random columns per row (fp32 values from a 255-entry codebook),
y = B x + 0.5 y with the library's AUTO path (the blocked column-band kernel
+ slab combine).  A step is one SpMV over one matrix.
To measure HBM rather than the 256 MiB Infinity Cache, steps rotate over
`--replicas` independent copies (matrix, x, y): 4 x 151 MB per rank.

N>1 (torchrun, one process per GPU): weak scaling -- every rank owns 2^20 rows
of a (N*2^20) x (N*2^20) matrix with global columns; a step is one RCCL
all-gather of x (xGMI) and the local SpMV.  Steps are independent products
(rotating replicas), so the all-gather of step k+1 runs beside the SpMV of step
k (--no-overlap: strictly one after the other).  `value` is the sum of all
ranks' algorithmic bytes divided by the max-over-ranks step time.

Algorithmic bytes per SpMV: 8*nnz + 4*(rows+1) + 4*cols + 8*rows.

Also reported, on the same JSON line:
  roofline      the SpMV alone: algorithmic bytes / mean SpMV time vs 8 TB/s.  N=1:
                HIP events around the replay of the captured graph of K SpMVs, on
                the stream it runs on (so the time per SpMV includes the gaps
                between kernels); N>1: HIP events around each sm_spmv call on its
                stream.  `traffic` from rocprofv3 PMC
                (profiles/traffic_<workload>_<layout>.json).
  cpu_baseline  rank 0, N=1: the oracle's same-order CSR SpMV (C) on the same
                matrix, over the box's CPU share (OpenMP, <= 16 threads; SURVEY
                §8d B2) with the 1-thread figure inside; ~15 s of CPU work.
  spmm          config 3 (same matrix, N=32 right-hand sides), GFLOP/s.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def spmv_bytes(nnz: int, rows: int, cols: int) -> int:
    return 8 * nnz + 4 * (rows + 1) + 4 * cols + 8 * rows


def spmm_bytes(nnz: int, rows: int, cols: int, n: int) -> int:
    return 8 * nnz + 4 * (rows + 1) + 4 * n * cols + 8 * n * rows


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


LAYOUTS = {0: "stream", 1: "exact", 2: "blocked", 3: "gather", 4: "band2", 5: "cband"}
KERNELS = {"stream": "spmv_stream_kernel",
           "exact": "spmv_xband_kernel (exact band layout)",
           "blocked": "spmv_xband_kernel (blocked band layout, slab combine fused)",
           "gather": "spmv_gband_kernel (column-ordered bands, x gathered, slab combine fused)",
           "band2": "spmv_band2_kernel (balanced bands, distributed slab combine)",
           "cband": "spmv_band2_kernel<CB> (balanced bands of 4-byte codebook words, "
                    "distributed slab combine)"}


def load_traffic(workload: str, layout: str):
    """HBM bytes per SpMV measured by rocprofv3 PMC (tools/pmc_traffic.py)."""
    p = os.path.join(ROOT, "profiles", f"traffic_{workload}_{layout}.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rows-per-rank", type=int, default=1 << 20)
    ap.add_argument("--per-row", type=int, default=16)
    ap.add_argument("--replicas", type=int, default=4)
    ap.add_argument("--algo", default="auto")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-spmm", action="store_true")
    ap.add_argument("--spmm-n", type=int, default=32)
    ap.add_argument("--no-rmat", action="store_true",
                    help="skip the config-4 line (R-MAT scale 24 SpMV, N = 1 only)")
    ap.add_argument("--rmat-scale", type=int, default=24)
    ap.add_argument("--no-graph", action="store_true",
                    help="N=1: launch each timed step from Python instead of replaying the K "
                         "steps as one captured HIP graph")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="development: one process builds rank 0's slice of a W-rank job "
                         "(R rows x R*W columns, x filled locally instead of all-gathered)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N>1: all-gather then SpMV per step, instead of the all-gather of "
                         "step k+1 in flight beside the SpMV of step k")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import sparsematrix_amd as smd
    from sparsematrix_amd import synth
    from sparsematrix_amd.distributed import allgather_spmv_pipelined

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world} (use torch.distributed.run)")
    # Development rehearsal only: SM_BENCH_DEVICE pins every rank to one GPU and
    # SM_BENCH_BACKEND=gloo replaces RCCL, so the N>1 code path can run on a one-GPU box.
    dev_index = int(os.environ.get("SM_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        backend = os.environ.get("SM_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    smd.load()

    if args.replicas < 1:
        raise SystemExit("--replicas must be >= 1")
    if world > 1 and not args.no_overlap and args.replicas < 2:
        raise SystemExit("--gpus N>1 overlaps the all-gather of step k+1 with the SpMV of step k, "
                         "which needs >= 2 replicas (distinct x buffers); use --replicas 2+ or "
                         "--no-overlap")
    R = args.rows_per_rank
    emu = args.emulate_world if world == 1 and args.emulate_world > 1 else 1
    C = R * world * emu                    # global columns (= global rows)
    per = args.per_row
    reps = []
    for k in range(args.replicas):
        seed = 2 + 1000 * k + 7919 * rank
        rp, ci, va = synth.uniform_rows_device(R, C, per, seed=seed, device=dev)
        M = smd.SparseMatrix.from_csr(rp, ci, va, C, device=dev_index)
        g = torch.Generator(device=dev).manual_seed(seed + 1)
        x_local = torch.rand(R, generator=g, device=dev) * 2 - 1
        x_full = (torch.empty(C, device=dev) if world > 1 else
                  torch.rand(C, generator=g, device=dev) * 2 - 1 if emu > 1 else x_local)
        y = torch.rand(R, generator=g, device=dev) * 2 - 1
        reps.append(dict(M=M, rp=rp, ci=ci, va=va, x_local=x_local, x_full=x_full, y=y))
        if k:
            del rp, ci, va
    nnz = R * per
    bytes_rank = spmv_bytes(nnz, R, C)
    torch.cuda.synchronize()

    def step(i, ev=None):
        r = reps[i % len(reps)]
        if world > 1:
            dist.all_gather_into_tensor(r["x_full"], r["x_local"])
        if ev is not None:
            ev[0].record()
        r["M"].spmv(r["x_full"], r["y"], 1.0, 0.5, algo=args.algo)
        if ev is not None:
            ev[1].record()

    # N > 1, default: steps are independent products (rotating replicas), so the
    # all-gather of step k+1 runs beside the SpMV of step k (distributed.py,
    # allgather_spmv_pipelined) -- still one all-gather per step, no other collective.
    overlap = world > 1 and not args.no_overlap

    def products(start, count, evs=None):
        for j in range(count):
            r = reps[(start + j) % len(reps)]

            def local(xf, yl, r=r, e=(evs[j] if evs is not None else None)):
                if e is not None:
                    e[0].record()
                r["M"].spmv(xf, yl, 1.0, 0.5, algo=args.algo)
                if e is not None:
                    e[1].record()
            yield (local, r["x_local"], r["x_full"], r["y"])

    if overlap:
        allgather_spmv_pipelined(products(0, args.warmup))
    else:
        for i in range(args.warmup):
            step(i)
    torch.cuda.synchronize()
    # N = 1: the K timed SpMVs are captured once into a HIP graph (capturing runs
    # nothing) and replayed as one launch, so the timed region holds the kernels
    # back to back with no Python / ctypes / per-call launch cost between them; HIP
    # events bracket the whole region on the stream the kernels run on.  N > 1:
    # every step (RCCL all-gather + SpMV) is launched eagerly, with events around
    # each SpMV.
    use_graph = world == 1 and not args.no_graph
    graph = None
    if use_graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for i in range(args.steps):
                step(args.warmup + i)
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if use_graph:
        events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))]
        t0 = time.perf_counter()
        events[0][0].record()
        graph.replay()
        events[0][1].record()
    else:
        events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.steps)]
        t0 = time.perf_counter()
        if overlap:
            allgather_spmv_pipelined(products(args.warmup, args.steps, events))
        else:
            for i in range(args.steps):
                step(args.warmup + i, events[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in events]
    if use_graph:   # one region of K SpMVs: per-SpMV time incl. the gaps between kernels
        kern_ms = [kern_ms[0] / args.steps]
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = 1e3 * elapsed / args.steps
    value = bytes_rank * world / (elapsed / args.steps) / 1e9
    kmean = float(np.mean(kern_ms))
    kmed = float(np.median(kern_ms))
    achieved = bytes_rank / (kmean * 1e-3) / 1e9
    workload = f"spmv_{R}x{C}_{per}_per_row"
    info = reps[0]["M"].info()
    layout = LAYOUTS[info["has_xband"]] if args.algo in ("auto", "xband") else "stream"
    traffic = load_traffic(workload, layout) if world == 1 else None
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
            "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
            "traffic": traffic,
            # the HBM bytes the kernel really moves (PMC) over its measured time
            "traffic_frac": (round(traffic / (kmean * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)
                             if traffic else None),
            "traffic_source": (f"profiles/traffic_{workload}_{layout}.json (rocprofv3 PMC, "
                               "FETCH_SIZE x calibration + WRITE_SIZE)" if traffic else None),
            "kernel": KERNELS[layout], "layout": layout,
            "xband_slabs": info["xband_slabs"], "xband_block_rows": info["xband_block_rows"],
            "kernel_ms_mean": round(kmean, 5), "kernel_ms_median": round(kmed, 5),
            "alg_bytes_per_launch": bytes_rank}

    # ---- SpMM (config 3) on replica 0, same ranks ---------------------------------
    spmm = None
    if not args.no_spmm:
        N = args.spmm_n
        r0 = reps[0]
        g = torch.Generator(device=dev).manual_seed(3)
        X = torch.rand((C, N), generator=g, device=dev) * 2 - 1
        Y = torch.rand((R, N), generator=g, device=dev) * 2 - 1
        for _ in range(3):
            r0["M"].spmm(X, Y, 1.0, 0.5)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(10)]
        for a, b in ev:
            a.record()
            r0["M"].spmm(X, Y, 1.0, 0.5)
            b.record()
        torch.cuda.synchronize()
        sm_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        sb = spmm_bytes(nnz, R, C, N)
        spmm = {"n_rhs": N, "ms": round(sm_ms, 4),
                "gflops": round(2.0 * nnz * N / (sm_ms * 1e-3) / 1e9, 1),
                "hbm_gbs": round(sb / (sm_ms * 1e-3) / 1e9, 1),
                "hbm_frac": round(sb / (sm_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                "kernel": "spmm_rowpanel2_kernel<8>", "mfma": "not used (fp32 SpMM at "
                "~2 flop/B is HBM/gather bound; see DESIGN.md)"}
        del X, Y

    # ---- R-MAT (config 4) on rank 0 at N = 1: AUTO on a Graph500 graph --------------
    rmat = None
    if world == 1 and rank == 0 and not args.no_rmat:
        try:   # a failure here must not cost the config-2 line
            from sparsematrix_amd import synth
            torch.cuda.synchronize()
            t_b = time.perf_counter()
            rrp, rci, rva = synth.rmat_device(args.rmat_scale, 16, seed=4)
            rn = 1 << args.rmat_scale
            t_g = time.perf_counter()
            RM = smd.SparseMatrix.from_csr(rrp, rci, rva, rn, device=dev_index)
            t_c = time.perf_counter()
            rinfo = RM.info()
            g = torch.Generator(device=dev).manual_seed(4)
            rx = torch.rand(rn, generator=g, device=dev) * 2 - 1
            ry = torch.rand(rn, generator=g, device=dev) * 2 - 1
            for _ in range(3):
                RM.spmv(rx, ry, 1.0, 0.5)
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(10)]
            for a, b in ev:
                a.record()
                RM.spmv(rx, ry, 1.0, 0.5)
                b.record()
            torch.cuda.synchronize()
            r_ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
            rnnz = int(rci.numel())
            rb = spmv_bytes(rnnz, rn, rn)
            kind = ("band kind %d" % rinfo["has_xband"] if rinfo["has_xband"]
                    else ("sorted sliced-ELL (%s) + long-row segments"
                          % ("4-byte column|codebook-id words" if rinfo["sell_codebook"] else "column + value")
                          if rinfo["sell_slices"] else "stream"))
            rmat = {"scale": args.rmat_scale, "rows": rn, "nnz": rnnz,
                    "max_row_nnz": rinfo["max_row_nnz"], "ms": round(r_ms, 4),
                    "alg_bytes": rb, "gbs": round(rb / (r_ms * 1e-3) / 1e9, 1),
                    "frac": round(rb / (r_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                    "kernel": kind + (", relabeled columns" if rinfo["col_relabel"] else ""),
                    "generate_s": round(t_g - t_b, 1), "build_s": round(t_c - t_g, 1),
                    "timing": "HIP events around each SpMV (median of 10, eager launches, "
                              "x permutation and finalize included)"}
            del RM, rrp, rci, rva, rx, ry
            torch.cuda.empty_cache()
        except Exception as exc:  # noqa: BLE001
            rmat = {"error": f"{type(exc).__name__}: {exc}"[:300]}

    # ---- CPU baseline (rank 0, N = 1) --------------------------------------------
    cpu = None
    if world == 1 and rank == 0 and not args.no_cpu:
        import oracle
        r0 = reps[0]
        rp = r0["rp"].cpu().numpy()
        ci = r0["ci"].cpu().numpy()
        va = r0["va"].cpu().numpy()
        x = r0["x_full"].cpu().numpy()
        y0 = r0["y"].cpu().numpy()
        threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)))

        def timed(fn, budget):
            fn()                                                # warm
            n_rep, t_cpu = 0, 0.0
            while t_cpu < budget and n_rep < 5000:
                c0 = time.perf_counter()
                fn()
                t_cpu += time.perf_counter() - c0
                n_rep += 1
            return n_rep, t_cpu

        n1, t1 = timed(lambda: oracle.csr_spmv(rp, ci, va, x, y0, 1.0, 0.5), args.cpu_seconds)
        nm, tm = timed(lambda: oracle.csr_spmv_mt(rp, ci, va, x, y0, 1.0, 0.5, threads=threads),
                       args.cpu_seconds / 2)
        cpu = {"value": round(bytes_rank * nm / tm / 1e9, 3), "unit": "GB/s", "cores": threads,
               "kind": "port",
               "sample": f"oracle same-order CSR SpMV (C, OpenMP over rows, {threads} threads) on "
                         f"the full config-2 matrix (replica 0), {nm} reps in {tm:.1f} s",
               "ms_per_spmv": round(1e3 * tm / nm, 3),
               "single_thread": {"value": round(bytes_rank * n1 / t1 / 1e9, 3), "unit": "GB/s",
                                 "cores": 1, "ms_per_spmv": round(1e3 * t1 / n1, 3),
                                 "sample": f"{n1} reps in {t1:.1f} s (the reference kernel is "
                                           f"single-threaded)"},
               "cpu": cpu_model(),
               "nproc": os.cpu_count()}

    if rank == 0:
        line = {
            "metric": "CSR SpMV effective HBM GB/s", "value": round(value, 1), "unit": "GB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": workload, "rows_per_rank": R, "cols": C, "nnz_per_rank": nnz,
                       "per_row": per, "replicas": args.replicas, "algo": args.algo,
                       "alpha": 1.0, "beta": 0.5, "launch": "hip_graph" if use_graph else "eager",
                       "parallelism": f"row-partition x{world}" + (
                           ", RCCL all-gather(x)" + (" of step k+1 overlapped with SpMV k"
                                                     if overlap else "") if world > 1 else ""),
                       **({"emulate_world": emu} if emu > 1 else {})},
            "roofline": roof, "cpu_baseline": cpu, "spmm": spmm, "rmat": rmat,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
