#!/bin/bash
# Round 5: same-box A/B of the band kernel before (build/ab_old: commit 120453c) and after the
# prune (the in-tree library), config 2 and its fp32-values sub-line, alternating runs.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
: > "$OUT/r5_prune_ab.txt"
for rep in 1 2 3; do
  for v in old new; do
    lib=$ROOT/sparsematrix_amd/libsparsematrix_amd.so
    [[ $v == old ]] && lib=$ROOT/build/ab_old/libsparsematrix_amd.so
    SM_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-spmm --no-rmat --no-config5 > "$OUT/r5_prune_$v.log" 2>&1 || { tail -20 "$OUT/r5_prune_$v.log"; exit 21; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], 'kernel_ms', r['kernel_ms'], 'fp32_kernel_ms', r.get('fp32_values',{}).get('kernel_ms'), 'ms_per_step', d['ms_per_step'])" "$OUT/r5_prune_$v.log" $v | tee -a "$OUT/r5_prune_ab.txt"
  done
done
