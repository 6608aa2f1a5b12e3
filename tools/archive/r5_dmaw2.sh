#!/bin/bash
# Round 5: phase profiles of dmaw (8 loaders) and dmaw4 (4 loaders), bench A/B against dma3.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
DEV=$ROOT/build/dev/libsparsematrix_amd.so
: > "$OUT/r5_dmaw_prof.txt"
for t in 4 8 9; do
  SM_LIB_PATH=$DEV SM_BAND_TALL=$t SM_BAND2_ABLATE=4096 timeout -k 10 120 python -u tools/cband_prof.py >> "$OUT/r5_dmaw_prof.txt" 2>&1 || { tail -20 "$OUT/r5_dmaw_prof.txt"; exit 21; }
done
grep prof "$OUT/r5_dmaw_prof.txt"
timeout -k 10 300 python -u -m pytest tests/test_gpu_band2.py -q -x --timeout 180 --timeout-method thread -k "dma3_config2 or vs_oracle" > "$OUT/r5_dmaw_tests.log" 2>&1 || { tail -30 "$OUT/r5_dmaw_tests.log"; exit 20; }
tail -1 "$OUT/r5_dmaw_tests.log"
: > "$OUT/r5_dmaw_ab.txt"
for t in 4 9 8 4 9 8; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-spmm --no-rmat --no-config5 --no-fp32-values --band-tall $t > "$OUT/r5_dmaw_$t.log" 2>&1 || { tail -20 "$OUT/r5_dmaw_$t.log"; exit 22; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('band_tall', sys.argv[2], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'], 'ms_per_step', d['ms_per_step'], 'build_s', d['config']['build_s'])" "$OUT/r5_dmaw_$t.log" $t | tee -a "$OUT/r5_dmaw_ab.txt"
done
