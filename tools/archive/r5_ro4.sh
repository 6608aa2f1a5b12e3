#!/bin/bash
# Round 5: row-owner kernel (groups of four chunks by stage, non-blocking loader): band tests,
# phase profile, bench A/B against dma3.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
DEV=$ROOT/build/dev/libsparsematrix_amd.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_band2.py -q -x --timeout 120 --timeout-method thread -k "10 or ro" > "$OUT/r5_ro4_tests.log" 2>&1 || { tail -40 "$OUT/r5_ro4_tests.log"; exit 20; }
tail -1 "$OUT/r5_ro4_tests.log"
: > "$OUT/r5_ro4.txt"
for a in 0 8 25; do
  SM_LIB_PATH=$DEV SM_BAND_TALL=10 SM_RO_PROF=1 SM_RO_ABLATE=$a timeout -k 10 120 python -u tools/cband_prof.py > "$OUT/r5_ro4_prof$a.log" 2>&1 || { tail -20 "$OUT/r5_ro4_prof$a.log"; exit 21; }
  grep "ro prof" "$OUT/r5_ro4_prof$a.log" | tail -1 | tee -a "$OUT/r5_ro4.txt"
done
for t in 4 10 4 10; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-spmm --no-rmat --no-config5 --no-fp32-values --band-tall $t > "$OUT/r5_ro4_$t.log" 2>&1 || { tail -20 "$OUT/r5_ro4_$t.log"; exit 22; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('band_tall', sys.argv[2], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'], 'layout', r['layout'])" "$OUT/r5_ro4_$t.log" $t | tee -a "$OUT/r5_ro4.txt"
done
