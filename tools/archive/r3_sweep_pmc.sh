#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only) over rank 0's slice
# of the 8-rank config-2 shape for KINDS (auto = the gather-band kind, sweep = column-swept
# row blocks; dev build).  Output: gpurun_out/swpmc_<kind>/g*/ + summary text.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp SM_LIB_PATH=$ROOT/build/dev/libsparsematrix_amd.so
cd /tmp || exit 1
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
G2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"
G3="TCC_HIT_sum TCC_MISS_sum"
G4="FETCH_SIZE"
G5="TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"
for K in ${KINDS:-auto sweep}; do
  OUT=$ROOT/gpurun_out/swpmc_$K; mkdir -p "$OUT"
  if [[ $K == auto ]]; then unset SM_XBAND_KIND; else export SM_XBAND_KIND=$K; fi
  i=0
  for g in "$G1" "$G2" "$G3" "$G4" "$G5"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $g --kernel-trace --output-format csv -d "$OUT/g$i" -o run -- python3 "$ROOT/bench.py" --emulate-world 8 --steps 5 --warmup 1 --replays 2 --no-cpu --no-spmm --no-rmat --no-graph > "$OUT/g$i.log" 2>&1 || { tail -20 "$OUT/g$i.log"; exit 31; }
  done
  python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$ROOT/gpurun_out/swpmc_$K.txt"
done
cat "$ROOT"/gpurun_out/swpmc_*.txt
