"""SpMM (config 3: 1M x 1M, 16 terms/row, N right-hand sides) A/B timing of the
row-panel kernels: the gather-pipelined kernel (default) against the
one-group-at-a-time kernel (SM_SPMM_OLD=1).  Run under `rocprofv3 --kernel-trace
--stats` for device times; the printed event times include host submission.

    python tools/spmm_ab.py [--n 32,64] [--reps 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--per-row", type=int, default=16)
    ap.add_argument("--n", default="32")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ab-env", default="SM_SPMM_OLD",
                    help="variable toggled 1 (\"old\") / 0 (\"new\"), e.g. SM_SPMM_NT")
    ap.add_argument("--algo", default="auto", help="sm_spmm algorithm of the env A/B (e.g. mfma)")
    ap.add_argument("--algos", default="",
                    help="compare sm_spmm algorithms instead, e.g. auto,mfma (old = the first)")
    args = ap.parse_args()

    import numpy as np
    import torch

    import sparsematrix_amd as smd
    from sparsematrix_amd import synth

    smd.load()
    dev = torch.device("cuda", 0)
    R = args.rows
    rp, ci, va = synth.uniform_rows_device(R, R, args.per_row, seed=2, device=dev)
    M = smd.SparseMatrix.from_csr(rp, ci, va, R)
    nnz = R * args.per_row
    out = []
    for N in (int(v) for v in args.n.split(",")):
        g = torch.Generator(device=dev).manual_seed(3)
        X = torch.rand((R, N), generator=g, device=dev) * 2 - 1
        Y0 = torch.rand((R, N), generator=g, device=dev) * 2 - 1
        res = {}
        algos = args.algos.split(",") if args.algos else None
        for old in ("1", "0"):
            algo = args.algo
            if algos:
                algo = algos[0] if old == "1" else algos[1]
            else:
                os.environ[args.ab_env] = old
            Y = Y0.clone()
            for _ in range(3):
                M.spmm(X, Y, 1.0, 0.5, algo=algo)
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.reps)]
            for a, b in ev:
                a.record()
                M.spmm(X, Y, 1.0, 0.5, algo=algo)
                b.record()
            torch.cuda.synchronize()
            ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
            Y = Y0.clone()
            M.spmm(X, Y, 1.0, 0.5, algo=algo)
            res[old] = (ms, Y.cpu().numpy().view(np.uint32))
        same = bool(np.array_equal(res["0"][1], res["1"][1]))
        line = {"ab_env": args.algos or args.ab_env, "n_rhs": N, "old_ms": round(res["1"][0], 4), "new_ms": round(res["0"][0], 4),
                "gflops_new": round(2.0 * nnz * N / (res["0"][0] * 1e-3) / 1e9, 1),
                "bit_identical": same}
        print(json.dumps(line), flush=True)
        out.append(line)
        del X, Y0, Y
    os.environ.pop(args.ab_env, None)


if __name__ == "__main__":
    main()
