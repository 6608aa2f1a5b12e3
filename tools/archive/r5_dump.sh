#!/bin/bash
# Per-tile timeline dump of the cband kernel (development build, SM_BAND2_ABLATE=2048).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
SM_B2_TS_DUMP=1 SM_LIB_PATH=$ROOT/build/dev/libsparsematrix_amd.so SM_BAND2_ABLATE=2048 timeout -k 10 120 python -u tools/cband_prof.py > "$OUT/r5_tile_dump.txt" 2>&1 || { tail -20 "$OUT/r5_tile_dump.txt"; exit 21; }
grep -c tile "$OUT/r5_tile_dump.txt"
