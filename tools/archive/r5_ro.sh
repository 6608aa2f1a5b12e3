#!/bin/bash
# Round 5: row-owner codebook bands (band_tall = 10): tests, then bench A/B against dma3.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_band2.py -q -x --timeout 120 --timeout-method thread -k "10 or ro" > "$OUT/r5_ro_tests.log" 2>&1 || { tail -40 "$OUT/r5_ro_tests.log"; exit 20; }
tail -1 "$OUT/r5_ro_tests.log"
: > "$OUT/r5_ro_ab.txt"
for t in 4 10 4 10; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-spmm --no-rmat --no-config5 --no-fp32-values --band-tall $t > "$OUT/r5_ro_$t.log" 2>&1 || { tail -20 "$OUT/r5_ro_$t.log"; exit 22; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('band_tall', sys.argv[2], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'], 'ms_per_step', d['ms_per_step'], 'build_s', d['config']['build_s'], 'layout', r['layout'])" "$OUT/r5_ro_$t.log" $t | tee -a "$OUT/r5_ro_ab.txt"
done
