#!/bin/bash
# SQ/LDS counters for one SpMV algorithm on config 2 (one rocprofv3 pass per group,
# --kernel-trace only).  Usage: ALGO=xband bash tools/pmc_kernel.sh, or PMC_CMD=<command>
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmck
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
CMD=${PMC_CMD:-"python3 $ROOT/tools/spmv_sweep.py --tiles 4096 --algos ${ALGO:-xband} --replicas 2 --rounds 1 --reps 4"}
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
G2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"
G3="SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_ANY"
G4="TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"
# PMC_GROUPS: other groups, ';'-separated (each within one pass's per-block limits)
if [[ -n "${PMC_GROUPS:-}" ]]; then IFS=';' read -ra GROUPS_ <<< "$PMC_GROUPS"; else GROUPS_=("$G1" "$G2" "$G3" "$G4"); fi
rm -rf "$OUT"/g*
i=0
for g in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $g --kernel-trace --output-format csv -d "$OUT/g$i" -o run -- $CMD > "$OUT/g$i.log" 2>&1 || { tail -20 "$OUT/g$i.log"; exit 31; }
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT"
