#!/bin/bash
# Ablations of the gather-band kernel on rank 0's slice of the 8-rank config-2 shape
# (2^20 x 2^23, bench.py --emulate-world 8) and on config 5's rank slice: SM_GBAND_ABLATE =
# 0 full, 1 no x gathers, 2 no apply, 4 no slab hand-off, 3 neither gathers nor apply
# (development build; results wrong except 0).  Median graph replay per SpMV.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT" || exit 1
for W in ${WORKLOADS:-config2}; do
  for A in ${ABLS:-0 1 2 4 3}; do
    if [[ $W == config2 ]]; then ARGS="--emulate-world 8 --steps 30 --warmup 3"; else ARGS="--workload config5 --emulate-world 8 --steps 10 --warmup 2 --replays 3"; fi
    SM_LIB_PATH=build/dev/libsparsematrix_amd.so SM_GBAND_ABLATE=$A timeout -k 10 300 python -u bench.py $ARGS --no-cpu --no-spmm --no-rmat > "$OUT/gba_${W}_$A.log" 2>&1 || { tail -5 "$OUT/gba_${W}_$A.log"; exit 1; }
    python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']; print(f\"{sys.argv[2]:8s} abl {sys.argv[3]}: {r['kernel_ms']*1e3:8.1f} us  {r['layout']}  slabs {r.get('xband_slabs')}\")" "$OUT/gba_${W}_$A.log" "$W" "$A"
  done
done
