#!/bin/bash
# Round 5: the merge path with its column-sorted staging stream (development switch
# SM_MERGE_STAGE=1): merge tests through the development build with the stream, then R-MAT 24
# and config 2 timings with and without it.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
DEV=$ROOT/build/dev/libsparsematrix_amd.so
SM_LIB_PATH=$DEV SM_MERGE_STAGE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_merge.py -q -x --timeout 240 --timeout-method thread > "$OUT/r5_mstage_tests.log" 2>&1 || { tail -30 "$OUT/r5_mstage_tests.log"; exit 20; }
tail -1 "$OUT/r5_mstage_tests.log"
: > "$OUT/r5_mstage_ab.txt"
for st in 1 0; do
  for w in rmat uniform; do
    SM_LIB_PATH=$DEV SM_MERGE_STAGE=$st timeout -k 10 400 python -u tools/spmv_sweep.py --workload $w --scale 24 --tiles "" --algos merge,auto --replicas 1 --rounds 3 > "$OUT/r5_mstage_$st$w.log" 2>&1 || { tail -20 "$OUT/r5_mstage_$st$w.log"; exit 21; }
    echo "STAGE=$st $w: $(grep -E '^  (merge|auto)' "$OUT/r5_mstage_$st$w.log" | tr -s ' ' | tr '\n' ';')" | tee -a "$OUT/r5_mstage_ab.txt"
  done
done
