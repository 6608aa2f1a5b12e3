#!/usr/bin/env python3
"""Turn the rocprofv3 PMC passes of tools/pmc.sh into HBM bytes per launch.

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE (KB) come from the L2's
memory-side request counters, and on gfx950 FETCH_SIZE reads 1/2 of the bytes
of a wide (16 B/lane) coalesced stream.  The correction factor is calibrated in
the same session on the microbench's 1 GiB float4 stream read (known bytes) and
applied to the kernel's FETCH_SIZE; WRITE_SIZE is used as is.  Caveat kept in
the output: the SpMV kernel also issues 4-byte gathers (x) whose FETCH_SIZE
calibration is not established; the figure is the wide-stream-corrected one.

  python tools/pmc_traffic.py gpurun_out/pmc <kernel-substring[,substring...]> <workload> \
      <layout> [alg_bytes]

One SpMV may be several kernels (the blocked band layout: the band kernel and the
slab combine): their per-dispatch averages are summed.
"""
from __future__ import annotations

import csv
import json
import os
import sys
from collections import defaultdict

csv.field_size_limit(1 << 30)


def per_dispatch(path: str, kernel_subs: str) -> dict[str, float]:
    """Per-dispatch average of each counter, summed over the listed kernels."""
    out: dict[str, float] = defaultdict(float)
    n = 0
    for sub in kernel_subs.split(","):
        vals = defaultdict(list)
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                if sub in row["Kernel_Name"]:
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
        for k, v in vals.items():
            if v:
                out[k] += sum(v) / len(v)
        n = max([n] + [len(v) for v in vals.values()])
    return dict(out) | {"_dispatches": n}


def find(base: str, tag: str) -> str:
    d = os.path.join(base, tag)
    for root, _, files in os.walk(d):
        for fn in files:
            if fn.endswith("counter_collection.csv"):
                return os.path.join(root, fn)
    raise FileNotFoundError(d)


def main():
    base, ksub, workload, layout = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
    alg = int(sys.argv[5]) if len(sys.argv) > 5 else None
    fetch = per_dispatch(find(base, "bench_FETCH_SIZE"), ksub)
    write = per_dispatch(find(base, "bench_WRITE_SIZE"), ksub)
    hitmiss = per_dispatch(find(base, "bench_TCC_HIT_sum_TCC_MISS_sum"), ksub)
    cal = per_dispatch(find(base, "micro_FETCH_SIZE"), "read_kernel")
    cal_bytes = float(1 << 30)
    factor = cal_bytes / (cal["FETCH_SIZE"] * 1024.0)
    fetch_b = fetch["FETCH_SIZE"] * 1024.0
    write_b = write["WRITE_SIZE"] * 1024.0
    hbm = fetch_b * factor + write_b
    hit = hitmiss.get("TCC_HIT_sum", 0.0)
    miss = hitmiss.get("TCC_MISS_sum", 0.0)
    out = {
        "workload": workload, "layout": layout, "kernels": ksub.split(","),
        "dispatches": fetch["_dispatches"],
        "fetch_size_bytes_raw": fetch_b, "write_size_bytes": write_b,
        "fetch_correction_factor": round(factor, 4),
        "calibration": "microbench read_kernel, 1 GiB float4 stream: FETCH_SIZE*1024*factor = 1 GiB",
        "hbm_bytes_per_launch": round(hbm), "alg_bytes_per_launch": alg,
        "traffic_over_alg": round(hbm / alg, 3) if alg else None,
        "l2_hit_rate": round(hit / (hit + miss), 4) if hit + miss else None,
        "note": ("x gathers are 4-byte accesses; their FETCH_SIZE calibration is not established"
                 if layout == "stream" else
                 "x is read in wide 16-byte slices (the calibrated access width)"),
    }
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                       f"traffic_{workload}_{layout}.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
