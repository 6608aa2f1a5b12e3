#!/bin/bash
# Round 5: ablations of the row-owner kernel (development build; results wrong): phase profile
# and bench kernel time per variant (0 full, 1 no DMA, 2 no x reads, 4 no sum reads/writes,
# 6 neither, 8 no apply, 16 no loader waits, 25 = 1+8+16).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
DEV=$ROOT/build/dev/libsparsematrix_amd.so
: > "$OUT/r5_ro_abl.txt"
for a in 0 1 2 4 6 8 16 25; do
  SM_LIB_PATH=$DEV SM_BAND_TALL=10 SM_RO_PROF=1 SM_RO_ABLATE=$a timeout -k 10 120 python -u tools/cband_prof.py > "$OUT/r5_ro_abl_prof$a.log" 2>&1 || { tail -20 "$OUT/r5_ro_abl_prof$a.log"; exit 21; }
  grep "ro prof" "$OUT/r5_ro_abl_prof$a.log" | tail -1 | tee -a "$OUT/r5_ro_abl.txt"
  SM_LIB_PATH=$DEV SM_RO_ABLATE=$a timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-spmm --no-rmat --no-config5 --no-fp32-values --band-tall 10 > "$OUT/r5_ro_abl$a.log" 2>&1 || { tail -20 "$OUT/r5_ro_abl$a.log"; exit 22; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('ABL', sys.argv[2], 'kernel_ms', r['kernel_ms'], 'layout', r['layout'])" "$OUT/r5_ro_abl$a.log" $a | tee -a "$OUT/r5_ro_abl.txt"
done
