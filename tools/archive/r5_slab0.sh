#!/bin/bash
# Round 5: slab-0 width A/B (development build, SM_BAND_SLAB0 permille) on the bench's
# config-2 line, alternating; then the band tests on the product build.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
DEV=$ROOT/build/dev/libsparsematrix_amd.so
: > "$OUT/r5_slab0_ab.txt"
for p in ${PERMILLES:-1000 930 900 960 1000 930 900 960}; do
  SM_LIB_PATH=$DEV SM_BAND_SLAB0=$p timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-spmm --no-rmat --no-config5 --no-fp32-values > "$OUT/r5_slab0_$p.log" 2>&1 || { tail -20 "$OUT/r5_slab0_$p.log"; exit 21; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('permille', sys.argv[2], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'], 'ms_per_step', d['ms_per_step'])" "$OUT/r5_slab0_$p.log" $p | tee -a "$OUT/r5_slab0_ab.txt"
done
timeout -k 10 120 ./build/xstream 50 c > "$OUT/r5_xstream_c.txt" 2>&1 && cat "$OUT/r5_xstream_c.txt" && timeout -k 10 600 python -u -m pytest tests/test_gpu_band2.py -q -x --timeout 180 --timeout-method thread > "$OUT/r5_band2_tests.log" 2>&1 || { tail -30 "$OUT/r5_band2_tests.log"; exit 22; }
tail -2 "$OUT/r5_band2_tests.log"
