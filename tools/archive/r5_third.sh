#!/bin/bash
# Round 5, third GPU session: the per-CU L2 -> LDS streaming ceiling (xstream f), the banded
# variants with more buffers, dma3's own phase profile and tile timeline (development build),
# and gcb on R-MAT 24 with its gathers ablated (development build).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 120 ./build/xstream 50 f > "$OUT/r5_xflow.txt" 2>&1 || { tail -20 "$OUT/r5_xflow.txt"; exit 21; }
cat "$OUT/r5_xflow.txt"
timeout -k 10 180 ./build/xstream 50 > "$OUT/r5_xstream3.txt" 2>&1 || { tail -20 "$OUT/r5_xstream3.txt"; exit 22; }
cat "$OUT/r5_xstream3.txt"
DEV=$ROOT/build/dev/libsparsematrix_amd.so
SM_LIB_PATH=$DEV SM_BAND2_ABLATE=4096 timeout -k 10 120 python -u tools/cband_prof.py > "$OUT/r5_dma3_prof.txt" 2>&1 || { tail -20 "$OUT/r5_dma3_prof.txt"; exit 23; }
cat "$OUT/r5_dma3_prof.txt"
SM_LIB_PATH=$DEV SM_BAND2_ABLATE=2048 timeout -k 10 120 python -u tools/cband_prof.py > "$OUT/r5_dma3_timeline.txt" 2>&1 || { tail -20 "$OUT/r5_dma3_timeline.txt"; exit 24; }
cat "$OUT/r5_dma3_timeline.txt"
for a in 1 3; do
  RMAT_GCB_NO_SHUFFLE=1 SM_LIB_PATH=$DEV SM_GCB_ABLATE=$a timeout -k 10 300 python -u tools/rmat_gcb_ab.py 24 0 > "$OUT/r5_rmat_gcb_abl$a.txt" 2>&1 || { tail -20 "$OUT/r5_rmat_gcb_abl$a.txt"; exit 25; }
  cat "$OUT/r5_rmat_gcb_abl$a.txt"
done
