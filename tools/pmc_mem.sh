#!/bin/bash
# Memory-pipeline counters (TA / TCP / TCC) for one SpMV algorithm on config 2, one
# rocprofv3 pass per group, --kernel-trace only.  Usage: ALGO=xband bash tools/pmc_mem.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmcm
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
CMD="python3 $ROOT/tools/spmv_sweep.py --tiles 4096 --algos ${ALGO:-xband} --replicas 2 --rounds 1 --reps 4"
G1="TA_BUSY_avr TA_BUSY_max TA_TA_BUSY_sum GRBM_GUI_ACTIVE"
G2="TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum"
G3="TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_NC_READ_REQ_sum"
G4="TCC_BUSY_avr TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum"
i=0
for g in "$G1" "$G2" "$G3" "$G4"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $g --kernel-trace --output-format csv -d "$OUT/g$i" -o run -- $CMD > "$OUT/g$i.log" 2>&1 || { tail -20 "$OUT/g$i.log"; exit 31; }
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT"
