#!/bin/bash
# Round 5: dmaw (8 loader waves, two 45 KiB windows, 48-chunk bands) against dma3 on config 2
# (bench line, alternating), its tile timeline, then the band tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_band2.py -q -x --timeout 180 --timeout-method thread -k "dma3_config2 or (vs_oracle and 8)" > "$OUT/r5_dmaw_tests.log" 2>&1 || { tail -30 "$OUT/r5_dmaw_tests.log"; exit 20; }
tail -2 "$OUT/r5_dmaw_tests.log"
: > "$OUT/r5_dmaw_ab.txt"
for t in 4 8 4 8; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-spmm --no-rmat --no-config5 --no-fp32-values --band-tall $t > "$OUT/r5_dmaw_$t.log" 2>&1 || { tail -20 "$OUT/r5_dmaw_$t.log"; exit 21; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('band_tall', sys.argv[2], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'], 'ms_per_step', d['ms_per_step'], 'build_s', d['config']['build_s'])" "$OUT/r5_dmaw_$t.log" $t | tee -a "$OUT/r5_dmaw_ab.txt"
done
SM_LIB_PATH=$ROOT/build/dev/libsparsematrix_amd.so SM_BAND_TALL=8 SM_BAND2_ABLATE=2048 timeout -k 10 120 python -u tools/cband_prof.py > "$OUT/r5_dmaw_timeline.txt" 2>&1 || { tail -20 "$OUT/r5_dmaw_timeline.txt"; exit 22; }
cat "$OUT/r5_dmaw_timeline.txt"
timeout -k 10 600 python -u -m pytest tests/test_gpu_band2.py -q -x --timeout 180 --timeout-method thread > "$OUT/r5_band2_tests2.log" 2>&1 || { tail -30 "$OUT/r5_band2_tests2.log"; exit 23; }
tail -2 "$OUT/r5_band2_tests2.log"
