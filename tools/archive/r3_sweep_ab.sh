#!/bin/bash
# A/B of the column-swept row blocks (SM_XBAND_KIND=sweep, dev build) against AUTO on rank
# 0's slice of the 8-rank config-2 shape (2^20 x 2^23) and of config 5 (2^23 x 2^26).
# Median graph replay per SpMV from bench.py's roofline object.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT" || exit 1
for W in ${WORKLOADS:-config2 config5}; do
  for K in ${KINDS:-auto sweep}; do
    if [[ $W == config2 ]]; then ARGS="--emulate-world 8 --steps 30 --warmup 3"; else ARGS="--workload config5 --emulate-world 8 --steps 10 --warmup 2 --replays 3"; fi
    E=(); [[ $K != auto ]] && E=(SM_XBAND_KIND=$K)
    env SM_LIB_PATH=build/dev/libsparsematrix_amd.so "${E[@]}" timeout -k 10 300 python -u bench.py $ARGS --no-cpu --no-spmm --no-rmat > "$OUT/sw_${W}_$K.log" 2>&1 || { tail -5 "$OUT/sw_${W}_$K.log"; exit 1; }
    python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']; print(f\"{sys.argv[2]:8s} {sys.argv[3]:6s}: {r['kernel_ms']*1e3:8.1f} us  {r['layout']}  frac {r['frac']}\")" "$OUT/sw_${W}_$K.log" "$W" "$K"
  done
done
