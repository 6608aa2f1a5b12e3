#!/usr/bin/env python3
"""bench.py -- CSR SpMV effective HBM GB/s on MI355X (BASELINE.json metric).

Workloads:
  config2 (default)  B is 2^20 x 2^20 per rank with exactly 16 distinct uniformly
                     random columns per row (fp32 values from a 255-entry codebook),
                     y = B x + 0.5 y with the library's AUTO layout.  N = 1: BASELINE
                     config 2.  N > 1: weak scaling -- every rank owns a 2^20-row slab
                     of an (N*2^20) x 2^20 matrix, i.e. exactly config 2's problem per
                     GPU, x (2^20) all-gathered from N parts (`--square`: the round-3
                     form, (N*2^20) x (N*2^20), whose per-rank x grows with N).
  config5            strong scaling: 2^26 x 2^26 (`--global-rows`), 16 columns per row,
                     rows split in N equal slices (8M rows x 64M columns per rank at
                     N = 8).  On one GPU, `--emulate-world W` builds rank 0's slice of a
                     W-rank job (x filled locally instead of all-gathered).
A step is one product.  N = 1 rotates over `--replicas` independent (matrix, x, y)
copies so the working set exceeds the 256 MiB Infinity Cache (HBM, not cache).
N > 1 (torchrun, one process per GPU): each step is one RCCL all-gather of x over
xGMI plus the local SpMV, through the library's C ABI (`sm_multi_*`,
sparsematrix_amd/csrc/multi.cpp); torch.distributed (gloo) only exchanges the RCCL
unique id and runs the barriers / max-over-ranks.  Steps are independent products,
so the all-gather of step k+1 runs beside the SpMV of step k (`sm_multi_spmv_batch`;
`--no-overlap`: one after the other).  `value` = the sum of all ranks' algorithmic
bytes / the max-over-ranks time per step.

Algorithmic bytes per SpMV: 8*nnz + 4*(rows+1) + 4*cols + 8*rows.

Also on the same JSON line:
  roofline      the dominant kernel: algorithmic bytes / SpMV time vs 8 TB/s.  N = 1:
                HIP events around the replay of the captured graph of the K timed
                SpMVs (per-SpMV time incl. the gaps between kernels), and the same
                over `--replays` further replays (median / min / max reported) plus K
                eager launches with events around each (a per-launch distribution).
                N > 1: the local SpMV alone, K launches with events (median).
                `traffic`: rocprofv3 PMC (profiles/traffic_<workload>_<layout>.json).
  allgather     N > 1: the all-gather alone (K launches, events, median), and the
                serial step (all-gather + SpMV) split by sm_multi's own events.
  cpu_baseline  rank 0, N = 1: the oracle's same-order CSR SpMV (C, OpenMP over rows)
                on the same matrix over every core this job may use (affinity and
                cgroup quota, stated), with the 1-thread figure; the reference-format
                twin (oracle/refmodel.c AddMatMat, 1 thread, what the reference runs) at
                config 1 and 16k^2; and R-MAT over all cores.  ~30 s of CPU work.
  spmm          config 3 (same matrix, N = 32 right-hand sides): GFLOP/s, HBM fraction,
                traffic and MFMA utilisation from PMC (profiles/), median of 20.
  rmat          config 4 (R-MAT scale 24) SpMV, median of 20; merge_path: the same matrix by
                SM_ALGO_MERGE, over the CSR arrays and with its staging copy.
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
PEAK_F32_TFLOPS = 157.3  # dense fp32 (vector = matrix rate on gfx950)


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


def available_cores() -> dict:
    """Cores this job may run on: the affinity mask, capped by the cgroup CPU quota."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    use = min(aff, quota) if quota else aff
    return {"use": use, "affinity": aff, "cgroup_quota": quota, "nproc": os.cpu_count()}


LAYOUTS = {0: "stream", 1: "exact", 2: "blocked", 3: "gather", 4: "band2", 5: "cband", 6: "gcb"}
KERNELS = {"stream": "spmv_stream_kernel",
           "sell": "spmv_sell_kernel / spmv_csell_kernel (sorted sliced-ELL)",
           "exact": "spmv_xband_kernel (exact band layout)",
           "blocked": "spmv_xband_kernel (blocked band layout, slab combine fused)",
           "gather": "spmv_gband_kernel (column-ordered bands, x gathered, slab combine fused)",
           "band2": "spmv_band2_kernel (balanced bands, distributed slab combine)",
           "cband": "spmv_band2_kernel<CB, dma3> (balanced bands of 4-byte codebook words, x staged "
                    "by a loader wave's LDS-DMA, distributed slab combine)",
           "ccsell": "spmv_ccsell_kernel (column-chunked sorted sliced-ELL)",
           "gcb": "spmv_gcb_kernel (gathered chunk bands: 2016-term bands, x gathered, rows' sums in LDS)",
           "sweep": "spmv_sweep_kernel (column-swept 256-row blocks, one wavefront each)"}


def layout_of(info: dict) -> str:
    if info.get("sweep_blocks"):
        return "sweep"
    if info["has_xband"]:
        return LAYOUTS[info["has_xband"]]
    if info.get("ccsell_chunks"):
        return "ccsell"
    return "sell" if info["sell_slices"] else "stream"


def load_json(name: str):
    p = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def load_traffic(workload: str, layout: str):
    """HBM bytes per SpMV measured by rocprofv3 PMC (tools/pmc_traffic.py)."""
    d = load_json(f"traffic_{workload}_{layout}.json")
    return d.get("hbm_bytes_per_launch") if d else None


def stats(ms: list) -> dict:
    a = np.asarray(ms, np.float64)
    return {"median": round(float(np.median(a)), 5), "min": round(float(a.min()), 5),
            "max": round(float(a.max()), 5), "n": int(a.size)}


def event_times(torch, fn, count: int) -> list:
    """`count` calls of fn(), a HIP event pair around each on the current stream."""
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(count)]
    for i, (a, b) in enumerate(ev):
        a.record()
        fn(i)
        b.record()
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in ev]


def launch_ranks(n: int) -> int:
    """torch.distributed.run with N local ranks on this very command line (a child
    process; nothing in this process has initialised the GPU)."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)]
    return subprocess.call(cmd + sys.argv[1:])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=("config2", "config5"), default="config2")
    ap.add_argument("--rows-per-rank", type=int, default=1 << 20, help="config2")
    ap.add_argument("--global-rows", type=int, default=1 << 26, help="config5")
    ap.add_argument("--per-row", type=int, default=16)
    ap.add_argument("--square", action="store_true",
                    help="config2 N > 1: (N*2^20) x (N*2^20) instead of (N*2^20) x 2^20")
    ap.add_argument("--replicas", type=int, default=0, help="0: 4 (config2) / 1 (config5)")
    ap.add_argument("--replays", type=int, default=10,
                    help="N=1: extra graph replays for the per-SpMV time distribution")
    ap.add_argument("--algo", default="auto")
    ap.add_argument("--layout", default="auto",
                    help="A/B: force the matrix layout (sm_build_opts.layout name, e.g. gcb, gather)")
    ap.add_argument("--band-tall", type=int, default=0,
                    help="A/B: sm_build_opts.band_tall (0/4 dma3, 6 wide) for the config-2 matrices")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
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
                    help="one process builds rank 0's slice of a W-rank job (x filled locally "
                         "instead of all-gathered)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N>1: all-gather then SpMV per step, instead of the all-gather of "
                         "step k+1 in flight beside the SpMV of step k")
    ap.add_argument("--no-config5", action="store_true",
                    help="skip the config-5 sub-line (2^26 x 2^26 strong scaling over the N ranks)")
    ap.add_argument("--c5-global-rows", type=int, default=1 << 26)
    ap.add_argument("--c5-steps", type=int, default=10)
    ap.add_argument("--no-fp32-values", action="store_true",
                    help="skip roofline.fp32_values (config 2 with arbitrary fp32 values)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` outside a launcher: start the N ranks ourselves (one
        # process per GPU) before anything here touches the GPU, and exit with their code.
        raise SystemExit(launch_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    import sparsematrix_amd as smd
    from sparsematrix_amd import synth
    from sparsematrix_amd.distributed import MultiContext

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world} (use torch.distributed.run)")
    # Development rehearsal of the N > 1 bookkeeping on a one-GPU box: SM_BENCH_REHEARSE=1
    # puts every rank on GPU 0 and moves x over the gloo group (RCCL refuses two ranks
    # on one GPU); the numbers are not a measurement.
    rehearse = world > 1 and os.environ.get("SM_BENCH_REHEARSE") == "1"
    dev_index = 0 if rehearse else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:   # control plane only: unique id, barriers, max over ranks
        dist.init_process_group("gloo")
    smd.load()

    emu = args.emulate_world if world == 1 and args.emulate_world > 1 else 1
    parts = world * emu
    if args.workload == "config2":
        R = args.rows_per_rank
        # Global columns: 2^20 (each rank's slab is config 2 itself; weak scaling of the
        # distribution), or with --square the global row count.
        C = R * parts if args.square else R
        seed0 = 2
        replicas = args.replicas or 4
    else:
        if args.global_rows % parts:
            raise SystemExit("--global-rows must split evenly over the ranks")
        C = args.global_rows
        R = C // parts
        seed0 = 5
        replicas = args.replicas or 1
    per = args.per_row
    if world > 1 and C % world:
        raise SystemExit("the columns must split evenly over the ranks (one all-gather)")

    t_build0 = time.perf_counter()
    gen_s = 0.0
    reps = []
    for k in range(replicas):
        seed = seed0 + 1000 * k + 7919 * rank
        t_g0 = time.perf_counter()
        rp, ci, va = synth.uniform_rows_device(R, C, per, seed=seed, device=dev)
        torch.cuda.synchronize()
        gen_s += time.perf_counter() - t_g0
        bopts = {} if args.layout == "auto" else dict(layout=args.layout)
        if args.band_tall:
            bopts["band_tall"] = args.band_tall
        M = smd.SparseMatrix.from_csr(rp, ci, va, C, device=dev_index, opts=bopts or None)
        g = torch.Generator(device=dev).manual_seed(seed + 1)
        x_local = torch.rand(C // world if world > 1 else R, generator=g, device=dev) * 2 - 1
        x_full = (None if world > 1 else
                  torch.rand(C, generator=g, device=dev) * 2 - 1 if emu > 1 else x_local)
        if world == 1 and emu == 1 and args.workload == "config5":
            x_full = torch.rand(C, generator=g, device=dev) * 2 - 1
        y = torch.rand(R, generator=g, device=dev) * 2 - 1
        reps.append(dict(M=M, rp=rp if k == 0 else None, ci=ci if k == 0 else None,
                         va=va if k == 0 else None, x_local=x_local, x_full=x_full, y=y))
        del rp, ci, va
    build_s = time.perf_counter() - t_build0
    nnz = R * per
    bytes_rank = spmv_bytes(nnz, R, C)
    torch.cuda.synchronize()
    info = reps[0]["M"].info()
    layout = layout_of(info) if args.algo in ("auto", "xband", "sell") else args.algo
    workload = (f"spmv_{R}x{C}_{per}_per_row" if args.workload == "config2"
                else f"config5_{C}x{C}_{per}_per_row_rank0of{parts}")

    ctx = None
    path = None
    nccl_group = None
    fallback = None
    if world > 1:
        uid = torch.zeros(128, dtype=torch.uint8)
        err = None
        if rank == 0:
            try:
                uid = torch.frombuffer(bytearray(MultiContext.unique_id()), dtype=torch.uint8).clone()
            except Exception as exc:  # noqa: BLE001
                err = exc
        dist.broadcast(uid, 0)
        if rehearse:   # RCCL cannot put two ranks on one GPU: the same C-ABI context over gloo
            from sparsematrix_amd.distributed import host_staged_allgather
            try:
                ctx = MultiContext.with_collective(reps[0]["M"], world, rank, host_staged_allgather())
            except Exception as exc:  # noqa: BLE001
                err = exc
        elif err is None and int(uid.sum()) != 0:
            try:
                ctx = MultiContext(reps[0]["M"], world, rank, bytes(uid.numpy().tobytes()))
            except Exception as exc:  # noqa: BLE001
                err = exc
        ok = torch.tensor([1 if ctx is not None else 0], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 1:
            coll = "host-staged gloo all-gather (rehearsal)" if rehearse else "ncclAllGather"
            path = f"sm_multi_spmv_batch (C ABI, {coll})" if not args.no_overlap \
                else f"sm_multi_spmv (C ABI, {coll})"
        else:
            # The C-ABI context failed on some rank: the same data path through torch's
            # RCCL group (all_gather_into_tensor + the local SpMV), reported as such.
            if ctx is not None:
                ctx.close()
                ctx = None
            fallback = f"{type(err).__name__}: {err}"[:300] if err else "failed on another rank"
            nccl_group = None if rehearse else dist.new_group(backend="nccl")
            for r in reps:
                r["x_full"] = torch.empty(C, device=dev)
            path = "torch.distributed all_gather_into_tensor (RCCL; sm_multi fallback)"

    overlap = world > 1 and not args.no_overlap

    def run_steps(start: int, count: int):
        """`count` products from step `start` on (replicas rotate)."""
        idx = [(start + j) % len(reps) for j in range(count)]
        if world == 1:
            for i in idx:
                r = reps[i]
                r["M"].spmv(r["x_full"], r["y"], 1.0, 0.5, algo=args.algo)
        elif ctx is None:   # fallback: torch's RCCL all-gather, then the local SpMV
            from sparsematrix_amd.distributed import allgather_spmv_pipelined

            def products():
                for i in idx:
                    r = reps[i]
                    yield (lambda xf, yl, r=r: r["M"].spmv(xf, yl, 1.0, 0.5, algo=args.algo),
                           r["x_local"], r["x_full"], r["y"])
            if overlap and len(reps) > 1:
                allgather_spmv_pipelined(products(), group=nccl_group)
            else:
                for f, xl, xf, yl in products():
                    dist.all_gather_into_tensor(xf, xl, group=nccl_group)
                    f(xf, yl)
        elif overlap:
            ctx.spmv_batch([reps[i]["x_local"] for i in idx], [reps[i]["y"] for i in idx],
                           1.0, 0.5, algo=args.algo, mats=[reps[i]["M"] for i in idx])
        else:
            for i in idx:   # one product per call: its all-gather, then its SpMV
                r = reps[i]
                ctx.spmv_batch([r["x_local"]], [r["y"]], 1.0, 0.5, algo=args.algo, mats=[r["M"]])

    run_steps(0, args.warmup)
    torch.cuda.synchronize()
    # N = 1: the K timed SpMVs are captured once into a HIP graph (capturing runs
    # nothing) and replayed as one launch, so the timed region holds the kernels back
    # to back with no Python / ctypes / per-call launch cost between them.
    use_graph = world == 1 and not args.no_graph
    graph = None
    if use_graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            run_steps(args.warmup, args.steps)
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    if use_graph:
        graph.replay()
    else:
        run_steps(args.warmup, args.steps)
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    region_ms = ev0.elapsed_time(ev1)
    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = 1e3 * elapsed / args.steps
    value = bytes_rank * world / (elapsed / args.steps) / 1e9

    # ---- distributions, outside the timed region ----------------------------------
    dist_info = {}
    if use_graph:
        per_replay = []
        for _ in range(max(1, args.replays)):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            graph.replay()
            b.record()
            torch.cuda.synchronize()
            per_replay.append(a.elapsed_time(b) / args.steps)
        dist_info["graph_replay_ms_per_spmv"] = stats([region_ms / args.steps] + per_replay)
        kern_ms = float(np.median([region_ms / args.steps] + per_replay))
    xs_local = None
    if world == 1:
        def one(i):
            r = reps[i % len(reps)]
            r["M"].spmv(r["x_full"], r["y"], 1.0, 0.5, algo=args.algo)
        eager = event_times(torch, one, args.steps)
        dist_info["eager_launch_ms"] = stats(eager)
        if not use_graph:
            kern_ms = float(np.median(eager))
    else:
        # the all-gather alone, the local SpMV alone, and the serial step split by events
        x_tmp = torch.empty(C, device=dev)
        if ctx is not None:
            ag = event_times(torch, lambda i: ctx.allgather(reps[i % len(reps)]["x_local"]), args.steps)
        else:
            ag = event_times(torch, lambda i: dist.all_gather_into_tensor(
                x_tmp, reps[i % len(reps)]["x_local"], group=nccl_group), args.steps)

        def local(i):
            r = reps[i % len(reps)]
            r["M"].spmv(x_tmp, r["y"], 1.0, 0.5, algo=args.algo)
        loc = event_times(torch, local, args.steps)
        dist_info["allgather_ms"] = stats(ag)
        dist_info["allgather_bytes_per_rank"] = 4 * C
        dist_info["allgather_gbs_per_rank"] = round(4 * C / (float(np.median(ag)) * 1e-3) / 1e9, 1)
        dist_info["local_spmv_ms"] = stats(loc)
        if ctx is not None:
            ctx.set_timing(True)
            split = []
            for i in range(args.steps):   # the context's own matrix (replica 0)
                ctx.spmv(reps[0]["x_local"], reps[0]["y"], 1.0, 0.5, algo=args.algo)
                split.append(ctx.last_times())
            ctx.set_timing(False)
            dist_info["serial_step_split_ms"] = {"allgather": stats([s[0] for s in split]),
                                                "spmv": stats([s[1] for s in split])}
        if fallback:
            dist_info["sm_multi_fallback"] = fallback
        kern_ms = float(np.median(loc))
        del x_tmp
    achieved = bytes_rank / (kern_ms * 1e-3) / 1e9
    traffic = load_traffic(workload, layout) if world == 1 else None
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
            "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
            "traffic": traffic,
            # the HBM bytes the kernel really moves (PMC) over its measured time
            "traffic_frac": (round(traffic / (kern_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)
                             if traffic else None),
            "traffic_source": (f"profiles/traffic_{workload}_{layout}.json (rocprofv3 PMC, "
                               "FETCH_SIZE x calibration + WRITE_SIZE)" if traffic else None),
            "kernel": KERNELS.get(layout, layout), "layout": layout,
            "xband_slabs": info["xband_slabs"], "xband_block_rows": info["xband_block_rows"],
            "kernel_ms": round(kern_ms, 5),
            "kernel_ms_source": ("median over graph replays (per SpMV incl. inter-kernel gaps)"
                                 if use_graph else "median of per-launch HIP events"),
            "alg_bytes_per_launch": bytes_rank, "distribution": dist_info}

    # ---- config 2 with arbitrary fp32 values (rank 0, N = 1), right after the headline, in
    # the same chip state (after the R-MAT leg it measured 3 us slower) ----
    if (world == 1 and emu == 1 and args.workload == "config2" and not args.no_fp32_values
            and reps[0]["rp"] is not None):
        try:
            roof["fp32_values"] = fp32_values_line(args, torch, reps, R, C, bytes_rank, dev, dev_index)
        except Exception as exc:  # noqa: BLE001
            roof["fp32_values"] = {"error": f"{type(exc).__name__}: {exc}"[:300]}

    # ---- SpMM (config 3) on replica 0 -----------------------------------------------
    spmm = None
    if not args.no_spmm and args.workload == "config2":
        N = args.spmm_n
        r0 = reps[0]
        g = torch.Generator(device=dev).manual_seed(3)
        X = torch.rand((C, N), generator=g, device=dev) * 2 - 1
        Y = torch.rand((R, N), generator=g, device=dev) * 2 - 1
        for _ in range(3):
            r0["M"].spmm(X, Y, 1.0, 0.5)
        torch.cuda.synchronize()
        sm_ms_list = event_times(torch, lambda i: r0["M"].spmm(X, Y, 1.0, 0.5), 20)
        sm_ms = float(np.median(sm_ms_list))
        sb = spmm_bytes(nnz, R, C, N)
        swl = f"spmm_{R}x{C}_{per}_per_row_n{N}"
        st = load_json(f"traffic_{swl}_rowpanel2.json")
        mf = load_json(f"mfma_{swl}_rowpanel2.json")
        spmm = {"n_rhs": N, "ms": round(sm_ms, 4), "ms_stats": stats(sm_ms_list),
                "gflops": round(2.0 * nnz * N / (sm_ms * 1e-3) / 1e9, 1),
                "flop_frac": round(2.0 * nnz * N / (sm_ms * 1e-3) / 1e12 / PEAK_F32_TFLOPS, 4),
                "alg_bytes": sb, "hbm_gbs": round(sb / (sm_ms * 1e-3) / 1e9, 1),
                "hbm_frac": round(sb / (sm_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                "traffic": st.get("hbm_bytes_per_launch") if st else None,
                "traffic_source": f"profiles/traffic_{swl}_rowpanel2.json" if st else None,
                "mfma_util": mf.get("mfma_util") if mf else None,
                "mfma_insts": mf.get("mfma_insts") if mf else None,
                "mfma_source": (f"profiles/mfma_{swl}_rowpanel2.json (rocprofv3 "
                                "SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE, SQ_INSTS_VALU_MFMA_F32)"
                                if mf else None),
                "kernel": "spmm_rowpanel2_kernel<8> (fp32 VALU, bit-exact; DESIGN.md §3.5)"}
        if N == 32:   # the matrix-core variant (SM_ALGO_MFMA), same matrix and panel
            try:
                for _ in range(3):
                    r0["M"].spmm(X, Y, 1.0, 0.5, algo="mfma")
                torch.cuda.synchronize()
                mm_list = event_times(torch, lambda i: r0["M"].spmm(X, Y, 1.0, 0.5, algo="mfma"), 20)
                mm = float(np.median(mm_list))
                mfm = load_json(f"mfma_{swl}_mfma.json")
                spmm["mfma_variant"] = {
                    "ms": round(mm, 4), "ms_stats": stats(mm_list),
                    "gflops": round(2.0 * nnz * N / (mm * 1e-3) / 1e9, 1),
                    "hbm_frac": round(sb / (mm * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                    "mfma_util": mfm.get("mfma_util") if mfm else None,
                    "mfma_insts": mfm.get("mfma_insts") if mfm else None,
                    "mfma_source": ("profiles/mfma_" + swl + "_mfma.json (rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES / "
                                    "GRBM_GUI_ACTIVE, SQ_INSTS_VALU_MFMA_F32 of spmm_mfma_lds_kernel<8>)"
                                    if mfm else None),
                    "kernel": "spmm_mfma_lds_kernel<8> (gathered X rows staged through LDS by LDS-DMA, "
                              "v_mfma_f32_16x16x4_f32 on 16-row tiles; within the sum|terms| bound, not "
                              "bit-exact; DESIGN.md §3.5)"}
            except Exception as exc:  # noqa: BLE001
                spmm["mfma_variant"] = {"error": f"{type(exc).__name__}: {exc}"[:200]}
        del X, Y

    # ---- R-MAT (config 4) on rank 0 at N = 1 ----------------------------------------
    rmat = None
    rmat_host = None
    if world == 1 and emu == 1 and rank == 0 and not args.no_rmat and args.workload == "config2":
        try:   # a failure here must not cost the config-2 line
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
            r_list = event_times(torch, lambda i: RM.spmv(rx, ry, 1.0, 0.5), 20)
            r_ms = float(np.median(r_list))
            rnnz = int(rci.numel())
            rb = spmv_bytes(rnnz, rn, rn)
            lay = layout_of(rinfo)
            rmat = {"scale": args.rmat_scale, "rows": rn, "nnz": rnnz,
                    "max_row_nnz": rinfo["max_row_nnz"], "ms": round(r_ms, 4),
                    "ms_stats": stats(r_list), "alg_bytes": rb,
                    "gbs": round(rb / (r_ms * 1e-3) / 1e9, 1),
                    "frac": round(rb / (r_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                    "layout": lay, "col_relabel": rinfo["col_relabel"],
                    "sell_codebook": rinfo["sell_codebook"],
                    "generate_s": round(t_g - t_b, 1), "build_s": round(t_c - t_g, 1),
                    "timing": "HIP events around each SpMV (median of 20 eager launches, x "
                              "permutation and finalize included)"}
            # north_star's merge-path row balancing (SM_ALGO_MERGE) on the same
            # matrix: over the CSR arrays, then with its column-sorted staging copy
            try:
                m_list = event_times(torch, lambda i: RM.spmv(rx, ry, 1.0, 0.5, algo="merge"), 20)
                t_m = time.perf_counter()
                RS = smd.SparseMatrix.from_csr(rrp, rci, rva, rn, device=dev_index, opts={"merge_stage": 1})
                ms_build = time.perf_counter() - t_m
                for _ in range(3):
                    RS.spmv(rx, ry, 1.0, 0.5, algo="merge")
                s_list = event_times(torch, lambda i: RS.spmv(rx, ry, 1.0, 0.5, algo="merge"), 20)
                m_ms, s_ms = float(np.median(m_list)), float(np.median(s_list))
                rmat["merge_path"] = {
                    "ms": round(m_ms, 4), "frac": round(rb / (m_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                    "staged_ms": round(s_ms, 4),
                    "staged_frac": round(rb / (s_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                    "merge_stage_built": RS.info()["merge_stage"], "staged_build_s": round(ms_build, 1),
                    "note": "SM_ALGO_MERGE, median of 20 eager launches; staged = sm_build_opts."
                            "merge_stage (terms gathered in column order per 2048-item slice)"}
                del RS
            except Exception as exc:  # noqa: BLE001
                rmat["merge_path"] = {"error": f"{type(exc).__name__}: {exc}"[:300]}
            if not args.no_cpu:
                rmat_host = (rrp.cpu().numpy(), rci.cpu().numpy(), rva.cpu().numpy(),
                             rx.cpu().numpy(), ry.cpu().numpy(), rb)
            del RM, rrp, rci, rva, rx, ry
            torch.cuda.empty_cache()
        except Exception as exc:  # noqa: BLE001
            rmat = {"error": f"{type(exc).__name__}: {exc}"[:300]}

    # ---- the headline's graph again, after the SpMM and R-MAT legs (how
    # much the chip's state after those legs moves a graph replay of the same SpMVs) ----------
    if use_graph and (spmm is not None or rmat is not None):
        again = []
        for _ in range(max(3, args.replays)):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            graph.replay()
            b.record()
            torch.cuda.synchronize()
            again.append(a.elapsed_time(b) / args.steps)
        roof["replay_after_legs_ms"] = stats(again)

    # ---- config 5: 2^26 x 2^26 strong scaling over the job's ranks ------------------
    config5 = None
    if args.workload == "config2" and emu == 1 and not args.no_config5:
        if ctx is not None:   # the config-2 products are done with: make room
            ctx.close()
            ctx = None
        for r in reps:
            r["M"] = None
        torch.cuda.empty_cache()
        try:
            config5 = config5_line(args, torch, dist, world, rank, dev, dev_index, rehearse)
        except Exception as exc:  # noqa: BLE001
            config5 = {"error": f"{type(exc).__name__}: {exc}"[:300]}
            if world > 1:
                raise

    # ---- CPU baseline (rank 0, N = 1) --------------------------------------------
    cpu = None
    if world == 1 and rank == 0 and not args.no_cpu and reps[0]["rp"] is not None:
        cpu = cpu_baseline(args, reps[0], bytes_rank, rmat_host)

    if rank == 0:
        line = {
            "metric": "CSR SpMV effective HBM GB/s", "value": round(value, 1), "unit": "GB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5), "higher_is_better": True,
            "scaling": "weak" if args.workload == "config2" else "strong",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": workload, "global_rows": R * parts, "rows_per_rank": R, "cols": C,
                       "nnz_per_rank": nnz,
                       "per_row": per, "replicas": replicas, "algo": args.algo,
                       "alpha": 1.0, "beta": 0.5, "launch": "hip_graph" if use_graph else "eager",
                       "build_s": round(build_s, 1),   # every replica: generation + layout build
                       "build_s_per_matrix": round(build_s / max(replicas, 1), 2),
                       "generate_s": round(gen_s, 2),   # of which the synthetic CSR generation
                       "layout_build_s_per_matrix": round((build_s - gen_s) / max(replicas, 1), 2),
                       "parallelism": f"row-partition x{world}" + (
                           f", {path}" + (": all-gather of step k+1 beside SpMV k"
                                          if overlap else "") if world > 1 else ""),
                       **({"emulate_world": emu} if emu > 1 else {})},
            "roofline": roof, "cpu_baseline": cpu, "spmm": spmm, "rmat": rmat, "config5": config5,
        }
        print(json.dumps(line), flush=True)
    if ctx is not None:
        ctx.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def fp32_values_line(args, torch, reps, R, C, bytes_rank, dev, dev_index) -> dict:
    """the headline's matrix with arbitrary fp32 values (no 255-entry
    codebook: AUTO takes the 8-byte band2 entries instead of cband's 4-byte words), two
    replicas of the same structure, the K SpMVs replayed as one graph like the headline."""
    import sparsematrix_amd as smd
    r0 = reps[0]
    mats = []
    for k in range(2):
        g = torch.Generator(device=dev).manual_seed(77 + k)
        va = torch.rand(r0["ci"].numel(), generator=g, device=dev) * 2 - 1
        mats.append((smd.SparseMatrix.from_csr(r0["rp"], r0["ci"], va, C, device=dev_index),
                     reps[k % len(reps)]["x_full"], torch.empty_like(reps[k % len(reps)]["y"]).uniform_(-1, 1)))
        del va
    info = mats[0][0].info()
    steps = args.steps

    def run():
        for j in range(steps):
            M, x, y = mats[j % 2]
            M.spmv(x, y, 1.0, 0.5)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        run()
    torch.cuda.synchronize()
    per = []
    for _ in range(max(3, args.replays)):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        graph.replay()
        b.record()
        torch.cuda.synchronize()
        per.append(a.elapsed_time(b) / steps)
    ms = float(np.median(per))
    ach = bytes_rank / (ms * 1e-3) / 1e9
    del graph, mats
    torch.cuda.empty_cache()
    return {"layout": layout_of(info), "kernel": KERNELS.get(layout_of(info)), "kernel_ms": round(ms, 5),
            "ms_stats": stats(per), "achieved": round(ach, 1), "frac": round(ach / PEAK_HBM_GBS, 4),
            "sample": "config 2's structure, values uniform fp32 (16.7 M distinct), 2 replicas, "
                      "median over graph replays of the K SpMVs"}


def config5_line(args, torch, dist, world, rank, dev, dev_index, rehearse) -> dict:
    """SURVEY §8(d) config 5 (BASELINE.json configs[4]): the 2^26 x 2^26 matrix, 16 distinct
    uniform columns per row (seed 5 + 7919 * rank per slice), row-split over the job's N
    ranks -- strong scaling.  One RCCL all-gather of x per product through the C ABI
    (sm_multi_spmv_batch; N = 1: the plain SpMV of the whole matrix), K products timed
    between barriers, max over ranks.  Bytes: 8 nnz + 4 (rows + N) + N * 4 cols
    + 8 rows summed over ranks, each rank reading all of x; frac = bytes / t / (N * 8 TB/s).
    Also per rank: the local SpMV alone (events, max over ranks of the medians) and the
    all-gather alone."""
    import sparsematrix_amd as smd
    from sparsematrix_amd import synth
    from sparsematrix_amd.distributed import MultiContext, host_staged_allgather
    C, per = args.c5_global_rows, args.per_row
    if C % world:
        return {"error": f"{C} rows do not split over {world} ranks"}
    R = C // world
    t_b = time.perf_counter()
    rp, ci, va = synth.uniform_rows_device(R, C, per, seed=5 + 7919 * rank, device=dev)
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t_b
    M = smd.SparseMatrix.from_csr(rp, ci, va, C, device=dev_index,
                                  opts=None if args.layout == "auto" else dict(layout=args.layout))
    del rp, ci, va
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t_b
    g = torch.Generator(device=dev).manual_seed(6 + rank)
    x_local = torch.rand(C // world, generator=g, device=dev) * 2 - 1
    y = torch.rand(R, generator=g, device=dev) * 2 - 1
    x_full = torch.rand(C, generator=g, device=dev) * 2 - 1
    ctx = None
    if world > 1:
        if rehearse:
            ctx = MultiContext.with_collective(M, world, rank, host_staged_allgather())
        else:
            uid = torch.zeros(128, dtype=torch.uint8)
            if rank == 0:
                uid = torch.frombuffer(bytearray(MultiContext.unique_id()), dtype=torch.uint8).clone()
            dist.broadcast(uid, 0)
            ctx = MultiContext(M, world, rank, bytes(uid.numpy().tobytes()))
    K = max(1, args.c5_steps)

    def run(count):
        if ctx is None:
            for _ in range(count):
                M.spmv(x_full, y, 1.0, 0.5)
        else:
            ctx.spmv_batch([x_local] * count, [y] * count, 1.0, 0.5)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
    run(2)
    barrier()
    t0 = time.perf_counter()
    run(K)
    barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    local = event_times(torch, lambda i: M.spmv(x_full, y, 1.0, 0.5), K)
    lm = torch.tensor([float(np.median(local))], dtype=torch.float64)
    ag = (event_times(torch, lambda i: ctx.allgather(x_local), K) if ctx is not None else None)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(lm, op=dist.ReduceOp.MAX)
    step_ms = 1e3 * float(el.item()) / K
    nnz = C * per
    bytes_total = 8 * nnz + 4 * (C + world) + world * 4 * C + 8 * C
    bytes_rank = 8 * R * per + 4 * (R + 1) + 4 * C + 8 * R
    value = bytes_total / (step_ms * 1e-3) / 1e9
    info = M.info()
    lay = layout_of(info)
    wl = f"config5_{C}x{C}_{per}_per_row_rank0of{world}"
    traffic = load_traffic(wl, lay)
    lms = float(lm.item())
    out = {"workload": f"config5_{C}x{C}_{per}_per_row", "ranks": world, "rows_per_rank": R,
           "scaling": "strong", "steps": K, "ms_per_step": round(step_ms, 4),
           "value": round(value, 1), "unit": "GB/s", "frac": round(value / (world * PEAK_HBM_GBS), 4),
           "alg_bytes_total": bytes_total, "alg_bytes_rank": bytes_rank,
           "local_spmv_ms_max_over_ranks": round(lms, 4), "local_spmv_ms_rank0": stats(local),
           "kernel_frac": round(bytes_rank / (lms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
           "layout": lay, "kernel": KERNELS.get(lay, lay), "build_s": round(build_s, 1), "generate_s": round(gen_s, 2),
           "layout_build_s": round(build_s - gen_s, 2),
           "traffic": traffic,
           "traffic_source": (f"profiles/traffic_{wl}_{lay}.json (rocprofv3 PMC)" if traffic else None),
           "path": ("one SpMV of the whole matrix per step" if ctx is None else
                    "sm_multi_spmv_batch: one all-gather of x per product (C ABI, "
                    + ("host-staged gloo" if rehearse else "ncclAllGather")
                    + "), all-gather k+1 beside SpMV k")}
    if ag is not None:
        out["allgather_ms"] = stats(ag)
        out["allgather_bytes_per_rank"] = 4 * C
    if ctx is not None:
        ctx.close()
    del M, x_local, x_full, y
    torch.cuda.empty_cache()
    return out


def cpu_baseline(args, r0, bytes_rank, rmat_host):
    """B2 (same-order CSR, all cores + 1 thread), B1 (the reference-format
    twin, 1 thread, config 1 and 16k^2), B3 (dense sgemv, config 1), B2 on R-MAT.  The oracle is the checker and
    this CPU baseline only; nothing of it runs in the timed GPU region."""
    import oracle
    from sparsematrix_amd import synth
    rp = r0["rp"].cpu().numpy()
    ci = r0["ci"].cpu().numpy()
    va = r0["va"].cpu().numpy()
    x = r0["x_full"].cpu().numpy()
    y0 = r0["y"].cpu().numpy()
    cores = available_cores()
    threads = cores["use"]

    def timed(fn, budget):
        fn()                                                # warm
        n_rep, t_cpu = 0, 0.0
        while t_cpu < budget and n_rep < 5000:
            c0 = time.perf_counter()
            fn()
            t_cpu += time.perf_counter() - c0
            n_rep += 1
        return n_rep, t_cpu

    sec = args.cpu_seconds
    n1, t1 = timed(lambda: oracle.csr_spmv(rp, ci, va, x, y0, 1.0, 0.5), sec)
    nm, tm = timed(lambda: oracle.csr_spmv_mt(rp, ci, va, x, y0, 1.0, 0.5, threads=threads), sec / 2)
    out = {"value": round(bytes_rank * nm / tm / 1e9, 3), "unit": "GB/s", "cores": threads,
           "kind": "port",
           "sample": f"oracle same-order CSR SpMV (C, OpenMP over rows, {threads} threads = every "
                     f"core this job may use) on the full config-2 matrix (replica 0), {nm} reps "
                     f"in {tm:.1f} s",
           "ms_per_spmv": round(1e3 * tm / nm, 3),
           "cores_detail": cores,
           "single_thread": {"value": round(bytes_rank * n1 / t1 / 1e9, 3), "unit": "GB/s",
                             "cores": 1, "ms_per_spmv": round(1e3 * t1 / n1, 3),
                             "sample": f"{n1} reps in {t1:.1f} s"},
           "cpu": cpu_model()}
    # B1: the reference-format twin (uint8 deltas + ids + 256-column panels, the
    # reference's AddMatMat op order, 1 thread): config 1 and 16k^2 at 0.1 %.
    b1 = {}
    table = synth.codebook()
    for name, n, dens, seed in (("config1_1024x1024_1pct", 1024, 0.01, 1),
                                ("16384x16384_0.1pct", 16384, 0.001, 6)):
        rng = np.random.default_rng(seed)
        live = rng.random((n, n)) < dens
        dm = np.where(live, rng.integers(0, 255, (n, n)), 255).astype(np.uint8)
        t_e = time.perf_counter()
        ref = oracle.RefModel(dm, n, n, n, table, 255, trans=True)
        enc_s = time.perf_counter() - t_e
        a = rng.uniform(-1, 1, n).astype(np.float32)
        c = rng.uniform(-1, 1, n).astype(np.float32)
        k, t_r = timed(lambda: ref.add_mat_mat(a, 1, n, c, n, 1.0, 0.5), min(2.0, sec / 4))
        nz = ref.nnz()
        ms = 1e3 * t_r / k
        b1[name] = {"ms": round(ms, 4), "nnz": int(nz),
                    "gbs": round(spmv_bytes(nz, n, n) / (ms * 1e-3) / 1e9, 3),
                    "encode_s": round(enc_s, 3), "reps": k}
        del dm, live, ref
    out["b1_reference_format_1thread"] = {
        "kind": "port", "cores": 1, "cases": b1,
        "sample": "oracle/refmodel.c AddMatMat on the reference's own format (m = 1, alpha 1, "
                  "beta 0.5), B = dense uint8 id matrix (Trans), codebook of 255 floats"}
    # B3: the dense baseline of the reference's harness (cblas_sgemv/sgemm on the dense
    # matrix, blas_test.h), config 1 only, through numpy's bundled OpenBLAS -- the only
    # OpenBLAS on the box (the reference's vendored "plus" builds are ARM-only).
    try:
        from threadpoolctl import threadpool_info, threadpool_limits
        blas = [i for i in threadpool_info() if i.get("user_api") == "blas"]
        rng = np.random.default_rng(1)
        dense = np.where(rng.random((1024, 1024)) < 0.01,
                         rng.uniform(-1, 1, (1024, 1024)), 0.0).astype(np.float32)
        xv = rng.uniform(-1, 1, 1024).astype(np.float32)
        yv = rng.uniform(-1, 1, 1024).astype(np.float32)
        with threadpool_limits(limits=1, user_api="blas"):
            k, t_r = timed(lambda: 0.5 * yv + dense @ xv, min(2.0, sec / 4))
        out["b3_dense_sgemv_config1_1thread"] = {
            "ms": round(1e3 * t_r / k, 4), "reps": k, "cores": 1,
            "blas": (blas[0].get("internal_api", "?") + " " + str(blas[0].get("version", "")))
            if blas else "unknown",
            "sample": "y = 0.5 y + A x, A the dense 1024 x 1024 fp32 matrix (1 % nonzero), numpy's BLAS"}
    except Exception as exc:  # noqa: BLE001
        out["b3_dense_sgemv_config1_1thread"] = {"unavailable": f"{type(exc).__name__}: {exc}"[:200]}
    if rmat_host is not None:
        rrp, rci, rva, rx, ry, rb = rmat_host
        k, t_r = timed(lambda: oracle.csr_spmv_mt(rrp, rci, rva, rx, ry, 1.0, 0.5, threads=threads),
                       sec / 2)
        out["rmat"] = {"ms_per_spmv": round(1e3 * t_r / k, 3), "cores": threads,
                       "gbs": round(rb * k / t_r / 1e9, 3), "reps": k,
                       "sample": "same-order CSR SpMV over the R-MAT scale-24 CSR"}
    return out


if __name__ == "__main__":
    main()
