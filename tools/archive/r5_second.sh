#!/bin/bash
# Round 5, second GPU session: the corrected x-stream microbench, the hand-off wrap test,
# then smoke, bench and its rocprofv3 stats.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 180 ./build/xstream 50 > "$OUT/r5_xstream2.txt" 2>&1 || { tail -20 "$OUT/r5_xstream2.txt"; exit 21; }
cat "$OUT/r5_xstream2.txt"
timeout -k 10 300 python -u -m pytest tests/test_gpu_band2.py -k "handoff_counter" -q --timeout 120 --timeout-method thread > "$OUT/r5_wrap_test.log" 2>&1 || { tail -30 "$OUT/r5_wrap_test.log"; exit 22; }
tail -2 "$OUT/r5_wrap_test.log"
STEPS=smoke,bench,prof bash tools/gpu_check.sh
timeout -k 10 500 python -u tools/rmat_gcb_ab.py 24 0 > "$OUT/r5_rmat_gcb_ab2.txt" 2>&1 || { tail -20 "$OUT/r5_rmat_gcb_ab2.txt"; exit 23; }
cat "$OUT/r5_rmat_gcb_ab2.txt"
