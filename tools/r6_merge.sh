#!/bin/bash
# Round 6: the merge path after the wave-scan join and the parallel fixup -- its tests
# (R-MAT 24 full size, a row over thousands of workgroups), R-MAT 24 timings of both plans, and
# the PMC traffic passes of the same command (tools/pmc.sh with PMC_CMD).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_merge.py -q -x --timeout 600 --timeout-method thread > "$OUT/r6_merge_tests.log" 2>&1 || { tail -40 "$OUT/r6_merge_tests.log"; exit 21; }
tail -n 2 "$OUT/r6_merge_tests.log"
for i in 1 2; do
  timeout -k 10 300 python -u tools/rmat_merge_run.py 20 > "$OUT/r6_merge_time$i.txt" 2>&1 || { tail -20 "$OUT/r6_merge_time$i.txt"; exit 22; }
  grep rmat24 "$OUT/r6_merge_time$i.txt"
done
rm -rf "$OUT/pmc"
RMAT_AUTO=0 PMC_CMD="python3 $ROOT/tools/rmat_merge_run.py 5" bash tools/pmc.sh || exit 23
