#!/bin/bash
# Round 5: merge-path items per thread (4 / 8 / 12 / 16; A/B builds under build/ipt*), config 2
# and R-MAT 24, event medians.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
: > "$OUT/r5_merge_ipt.txt"
for v in 4 8 12 16; do
  lib=$ROOT/sparsematrix_amd/libsparsematrix_amd.so
  [[ $v != 8 ]] && lib=$ROOT/build/ipt$v/libsparsematrix_amd.so
  for w in uniform rmat; do
    SM_LIB_PATH=$lib timeout -k 10 400 python -u tools/spmv_sweep.py --workload $w --scale 24 --tiles "" --algos merge --replicas 1 --rounds 3 > "$OUT/r5_merge_ipt_$v_$w.log" 2>&1 || { tail -20 "$OUT/r5_merge_ipt_$v_$w.log"; exit 21; }
    echo "IPT $v $w $(grep merge "$OUT/r5_merge_ipt_$v_$w.log" | tail -1)" | tee -a "$OUT/r5_merge_ipt.txt"
  done
done
