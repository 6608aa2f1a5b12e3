#!/bin/bash
# TCP/TCC latency and stall counters of config 2's cband kernel: the in-tree library,
# then the dev library (build/dev, -DSM_DEV) under each SM_BAND2_ABLATE value in ABLS.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export PMC_GROUPS="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum;TCP_TCP_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum;TCC_HIT_sum TCC_MISS_sum TCC_LATENCY_FIFO_FULL_sum GRBM_GUI_ACTIVE;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES TA_TA_BUSY_sum TD_TD_BUSY_sum TD_TC_STALL_sum"
export PMC_CMD="python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu --no-spmm --no-rmat"
for v in tree ${ABLS:-}; do
  if [[ $v == tree ]]; then unset SM_LIB_PATH SM_BAND2_ABLATE; else export SM_LIB_PATH=$ROOT/build/dev/libsparsematrix_amd.so SM_BAND2_ABLATE=$v; fi
  echo "=== $v"
  bash "$ROOT/tools/pmc_kernel.sh" 2>&1 | grep -A40 spmv_band2 || exit 31
done
# MALL residency: one replica (entries + x + y + partials ~ 100 MB stay in the 256 MiB
# Infinity Cache across SpMVs) against the default four.
if [[ -n "${MALL:-}" ]]; then
  unset SM_LIB_PATH SM_BAND2_ABLATE
  for r in 1 4; do
    timeout -k 10 300 python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu --no-spmm --no-rmat --replicas $r > "$OUT/mall_r$r.log" 2>&1 || exit 32
    echo "replicas $r: $(grep '^{' "$OUT/mall_r$r.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms"], d["roofline"]["distribution"])')"
  done
fi
