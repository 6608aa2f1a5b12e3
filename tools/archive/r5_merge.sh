#!/bin/bash
# Round 5: merge-path SpMV (SM_ALGO_MERGE): its tests, then config 2 and R-MAT 24 timings against
# AUTO and the stream kernel (event medians, tools/spmv_sweep.py) and rocprofv3 kernel stats.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_merge.py -q -x --timeout 240 --timeout-method thread > "$OUT/r5_merge_tests.log" 2>&1 || { tail -40 "$OUT/r5_merge_tests.log"; exit 20; }
tail -1 "$OUT/r5_merge_tests.log"
timeout -k 10 300 python -u tools/spmv_sweep.py --workload uniform --tiles "" --algos merge,stream,auto --replicas 2 --rounds 3 > "$OUT/r5_merge_uniform.txt" 2>&1 || { tail -20 "$OUT/r5_merge_uniform.txt"; exit 21; }
tail -6 "$OUT/r5_merge_uniform.txt"
timeout -k 10 400 python -u tools/spmv_sweep.py --workload rmat --scale 24 --tiles "" --algos merge,stream,auto --replicas 1 --rounds 3 > "$OUT/r5_merge_rmat.txt" 2>&1 || { tail -20 "$OUT/r5_merge_rmat.txt"; exit 22; }
tail -6 "$OUT/r5_merge_rmat.txt"
rm -rf "$OUT/merge_stats"
( cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/merge_stats" -o run -- \
    python3 "$ROOT/tools/spmv_sweep.py" --workload uniform --tiles "" --algos merge --replicas 2 --rounds 2 ) > "$OUT/merge_stats.log" 2>&1 || { tail -20 "$OUT/merge_stats.log"; exit 23; }
find "$OUT/merge_stats" -name '*kernel_stats.csv' -exec grep -h "merge" {} \; | cut -c1-80,180-300
