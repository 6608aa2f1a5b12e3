#!/bin/bash
# Round 5, first GPU session: the x-stream microbench (tools/xstream.hip), then the whole
# GPU suite, smoke, the bench line and its rocprofv3 stats (tools/gpu_check.sh).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 180 ./build/xstream 50 > "$OUT/r5_xstream.txt" 2>&1 || { tail -20 "$OUT/r5_xstream.txt"; exit 21; }
cat "$OUT/r5_xstream.txt"
bash tools/gpu_check.sh
timeout -k 10 400 python -u tools/rmat_gcb_ab.py 24 0 > "$OUT/r5_rmat_gcb_ab.txt" 2>&1 || { tail -20 "$OUT/r5_rmat_gcb_ab.txt"; exit 22; }
cat "$OUT/r5_rmat_gcb_ab.txt"
