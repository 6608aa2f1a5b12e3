#!/bin/bash
# Round 6: counters (after dropping the dead lanes' LDS atomics) of the reference-format kernels on 16384^2 at 0.1 %, m = 1:
# kernel-trace stats, then SQ / LDS counter passes (tools/pmc_kernel.sh).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export NATIVE_CASES=16384 NATIVE_M=1 NATIVE_ALGOS=native TMPDIR=/tmp
timeout -k 10 200 python3 "$ROOT/tools/native_bench.py" > "$OUT/r6_native_bench.txt" 2>&1 || { tail -20 "$OUT/r6_native_bench.txt"; exit 20; }
cat "$OUT/r6_native_bench.txt"
rm -rf "$OUT/nstat"
( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/nstat" -o run -- python3 "$ROOT/tools/native_bench.py" ) > "$OUT/nstat.log" 2>&1 || { tail -20 "$OUT/nstat.log"; exit 21; }
find "$OUT/nstat" -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-220
PMC_CMD="python3 $ROOT/tools/native_bench.py" \
PMC_GROUPS="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT;SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE;SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE" \
  timeout -k 10 600 bash "$ROOT/tools/pmc_kernel.sh" > "$OUT/r6_native_pmc.txt" 2>&1 || { tail -20 "$OUT/r6_native_pmc.txt"; exit 22; }
cat "$OUT/r6_native_pmc.txt"
