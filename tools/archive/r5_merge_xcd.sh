#!/bin/bash
# Round 5: merge path, XCD-contiguous slice runs (development switch SM_MERGE_XCD=1) against the
# default round-robin, staging copy on: merge tests with the switch, then R-MAT 24 and config 2.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
DEV=$ROOT/build/dev/libsparsematrix_amd.so
SM_LIB_PATH=$DEV SM_MERGE_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_merge.py -q -x --timeout 240 --timeout-method thread > "$OUT/r5_mxcd_tests.log" 2>&1 || { tail -30 "$OUT/r5_mxcd_tests.log"; exit 20; }
tail -1 "$OUT/r5_mxcd_tests.log"
: > "$OUT/r5_mxcd_ab.txt"
for rep in 1 2; do
  for xm in 1 0; do
    for w in rmat uniform; do
      SM_LIB_PATH=$DEV SM_MERGE_XCD=$xm timeout -k 10 400 python -u tools/spmv_sweep.py --workload $w --scale 24 --tiles "" --algos merge --replicas 1 --rounds 3 --opts '{"merge_stage": 1}' > "$OUT/r5_mxcd_$xm$w.log" 2>&1 || { tail -20 "$OUT/r5_mxcd_$xm$w.log"; exit 21; }
      echo "SM_MERGE_XCD=$xm $w: $(grep -E '^  merge' "$OUT/r5_mxcd_$xm$w.log" | tr -s ' ')" | tee -a "$OUT/r5_mxcd_ab.txt"
    done
  done
done
