#!/bin/bash
# Round 5: phase profile of the row-owner kernel (band_tall = 10) at entry depth 3 and 6,
# then bench timing of both depths through the development library.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
DEV=$ROOT/build/dev/libsparsematrix_amd.so
: > "$OUT/r5_ro_prof.txt"
for ae in 3 6; do
  echo "AE=$ae" >> "$OUT/r5_ro_prof.txt"
  SM_LIB_PATH=$DEV SM_BAND_TALL=10 SM_RO_PROF=1 SM_RO_AE=$ae timeout -k 10 120 python -u tools/cband_prof.py >> "$OUT/r5_ro_prof.txt" 2>&1 || { tail -20 "$OUT/r5_ro_prof.txt"; exit 21; }
done
grep -E "AE=|prof" "$OUT/r5_ro_prof.txt"
: > "$OUT/r5_ro_ab2.txt"
for ae in 3 6; do
  SM_LIB_PATH=$DEV SM_RO_AE=$ae timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-spmm --no-rmat --no-config5 --no-fp32-values --band-tall 10 > "$OUT/r5_ro_ae$ae.log" 2>&1 || { tail -20 "$OUT/r5_ro_ae$ae.log"; exit 22; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('AE', sys.argv[2], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'], 'layout', r['layout'])" "$OUT/r5_ro_ae$ae.log" $ae | tee -a "$OUT/r5_ro_ab2.txt"
done
