#!/bin/bash
# Round 5 evidence session: MFMA counters of both SpMM kernels,
# PMC traffic of config 5 on one GPU (gcb), and the 2-rank C-ABI rehearsal on the current
# weak-scaled workload.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
bash tools/pmc_mfma.sh || exit 31
PMC_CMD="python3 $ROOT/bench.py --workload config5 --steps 3 --warmup 1 --no-cpu" bash tools/pmc.sh || exit 32
cd "$ROOT" || exit 1
SM_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu --no-spmm --no-rmat > "$OUT/r5_rehearse_2rank.log" 2>&1 || { tail -20 "$OUT/r5_rehearse_2rank.log"; exit 33; }
tail -1 "$OUT/r5_rehearse_2rank.log"
