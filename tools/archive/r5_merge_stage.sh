#!/bin/bash
# Round 5: the merge path with its column-sorted staging copy (sm_build_opts.merge_stage):
# merge tests (both plans, bit-identical), then R-MAT 24 and config 2 timings with and without it.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_merge.py tests/test_capi_cpu.py -q -x --timeout 240 --timeout-method thread > "$OUT/r5_mstage_tests.log" 2>&1 || { tail -30 "$OUT/r5_mstage_tests.log"; exit 20; }
tail -1 "$OUT/r5_mstage_tests.log"
: > "$OUT/r5_mstage_ab.txt"
for st in 1 0; do
  for w in rmat uniform; do
    timeout -k 10 400 python -u tools/spmv_sweep.py --workload $w --scale 24 --tiles "" --algos merge,auto --replicas 1 --rounds 3 --opts "{\"merge_stage\": $st}" > "$OUT/r5_mstage_$st$w.log" 2>&1 || { tail -20 "$OUT/r5_mstage_$st$w.log"; exit 21; }
    echo "merge_stage=$st $w: $(grep -E '^  (merge|auto)' "$OUT/r5_mstage_$st$w.log" | tr -s ' ' | tr '\n' ';')" | tee -a "$OUT/r5_mstage_ab.txt"
  done
done
