"""Development: SpMV kernel time when a few CUs are busy with other kernels (as RCCL's
all-gather would be during the overlapped multi-GPU step).  Side streams run
torch.cuda._sleep (one workgroup each) while the SpMV launches on the main stream.

    python tools/cu_contention.py [--busy 0,1,3] [--sleep-us 60]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--busy", default="0,1,3")
    ap.add_argument("--sleep-us", type=float, default=60.0)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch

    import sparsematrix_amd as smd
    from sparsematrix_amd import synth
    smd.load()
    dev = torch.device("cuda", 0)
    R = 1 << 20
    reps = []
    for k in range(4):
        rp, ci, va = synth.uniform_rows_device(R, R, 16, seed=2 + k, device=dev)
        reps.append((smd.SparseMatrix.from_csr(rp, ci, va, R), torch.rand(R, device=dev),
                     torch.rand(R, device=dev)))
    main_s = torch.cuda.current_stream()
    side = [torch.cuda.Stream() for _ in range(3)]
    # calibrate _sleep cycles -> us
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); torch.cuda._sleep(1_000_000); e1.record(); torch.cuda.synchronize()
    cyc = int(1_000_000 * args.sleep_us / 1e3 / e0.elapsed_time(e1))
    out = {}
    for nb in (int(v) for v in args.busy.split(",")):
        ts = []
        for i in range(args.reps):
            M, x, y = reps[i % 4]
            torch.cuda.synchronize()
            for s in side[:nb]:
                with torch.cuda.stream(s):
                    torch.cuda._sleep(cyc)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(main_s)
            M.spmv(x, y, 1.0, 0.5)
            b.record(main_s)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        out[f"busy_cus_{nb}"] = round(float(np.median(ts)) * 1e3, 1)
    out["sleep_us"] = args.sleep_us
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
