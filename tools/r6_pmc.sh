#!/bin/bash
# Round 6 record, second half: PMC traffic of the bench's config-2 kernel (tools/pmc.sh), the
# config-3 column-ordered pull experiment (build/spmm_colwin: its own check and time, then the
# same PMC passes), and the 2-rank rehearsal of the N > 1 bookkeeping on GPU 0.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
rm -rf "$OUT/pmc" "$OUT/pmc_colwin"
BENCH_ARGS="--no-config5 --no-fp32-values" bash tools/pmc.sh || exit $?
timeout -k 10 300 ./build/spmm_colwin 10 > "$OUT/r6_colwin.txt" 2>&1 || { tail -5 "$OUT/r6_colwin.txt"; exit 31; }
cat "$OUT/r6_colwin.txt"
PMC_OUT=$OUT/pmc_colwin PMC_CMD="$ROOT/build/spmm_colwin 3" bash tools/pmc.sh || exit $?
SM_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu --no-spmm --no-rmat > "$OUT/r6f_rehearse.log" 2>&1 || { tail -20 "$OUT/r6f_rehearse.log"; exit 33; }
grep '^{' "$OUT/r6f_rehearse.log" | tail -1 > "$OUT/r6f_rehearse_line.json"; cut -c1-300 "$OUT/r6f_rehearse_line.json"
echo "r6_pmc done"
