#!/bin/bash
# Round 4: SQ/LDS/TA counters of the dma3 cband kernel on config 2 (same groups as
# profiles/r03b_pmc_cband.txt, one rocprofv3 pass per group).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$ROOT/gpurun_out"
PMC_CMD="python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu --no-spmm --no-rmat --no-config5 --no-fp32-values" \
  bash "$ROOT/tools/pmc_kernel.sh" > "$ROOT/gpurun_out/r4_pmck.txt" 2>&1 || { tail -20 "$ROOT/gpurun_out/r4_pmck.txt"; exit 4; }
grep -A24 spmv_band2 "$ROOT/gpurun_out/r4_pmck.txt"
