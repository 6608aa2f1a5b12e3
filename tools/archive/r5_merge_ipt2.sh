#!/bin/bash
# Round 5: merge items per thread (SM_MERGE_IPT 4 / 6 / 8 / 16 / 32; development builds build/dev_iN,
# build/dev for 8; VARIANTS picks them), staging stream on: merge tests, then R-MAT 24 and config 2.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
: > "$OUT/r5_mipt_ab.txt"
for v in ${VARIANTS:-dev_i4 dev_i6 dev}; do
  L=$ROOT/build/$v/libsparsematrix_amd.so
  ipt=${v#dev_i}; [[ $v == dev ]] && ipt=8
  SM_MERGE_IPT=$ipt SM_LIB_PATH=$L SM_MERGE_STAGE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_merge.py -q -x --timeout 240 --timeout-method thread > "$OUT/r5_mipt_t_$v.log" 2>&1 || { tail -30 "$OUT/r5_mipt_t_$v.log"; exit 20; }
  echo "$v tests: $(tail -1 "$OUT/r5_mipt_t_$v.log")" | tee -a "$OUT/r5_mipt_ab.txt"
  for w in rmat uniform; do
    SM_LIB_PATH=$L SM_MERGE_STAGE=1 timeout -k 10 400 python -u tools/spmv_sweep.py --workload $w --scale 24 --tiles "" --algos merge --replicas 1 --rounds 3 > "$OUT/r5_mipt_$v$w.log" 2>&1 || { tail -20 "$OUT/r5_mipt_$v$w.log"; exit 21; }
    echo "$v $w: $(grep -E '^  merge' "$OUT/r5_mipt_$v$w.log" | tr -s ' ')" | tee -a "$OUT/r5_mipt_ab.txt"
  done
done
