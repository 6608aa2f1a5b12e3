#!/bin/bash
# Round 5: two-buffer x-stream variants with entries further ahead and a simulated apply.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 150 ./build/xstream 50 b > "$OUT/r5_xstream_b.txt" 2>&1 || { tail -20 "$OUT/r5_xstream_b.txt"; exit 21; }
cat "$OUT/r5_xstream_b.txt"
