#!/bin/bash
# Round 6: early publish of the rows the last band does not touch (loader wave; dev_e) against
# everything in the epilogue (dev_n: -DSM_B2_EARLY=0): bit-exact check, tile timelines, alternating
# bench A/B; then the band and device-builder tests on the product build.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
lib() { echo "$ROOT/build/dev_$1/libsparsematrix_amd.so"; }
SM_LIB_PATH=$(lib e) timeout -k 10 300 python -u tools/handoff_check.py > "$OUT/r6_check_e.txt" 2>&1 || { tail -20 "$OUT/r6_check_e.txt"; exit 21; }
grep -v amdgpu.ids "$OUT/r6_check_e.txt"
for v in n e; do
  SM_B2_TS_DUMP=1 SM_LIB_PATH=$(lib $v) SM_BAND2_PROF=2 timeout -k 10 150 python -u tools/cband_prof.py > "$OUT/r6_tl4_$v.txt" 2>&1 || { tail -20 "$OUT/r6_tl4_$v.txt"; exit 22; }
  echo "== $v"; grep -v "^  tile" "$OUT/r6_tl4_$v.txt" | tail -n 9
done
: > "$OUT/r6_early_ab.txt"
for i in 1 2 3; do
  for v in n e; do
    SM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 \
      --no-cpu --no-spmm --no-rmat --no-config5 > "$OUT/r6_eab_$v$i.log" 2>&1 || { tail -20 "$OUT/r6_eab_$v$i.log"; exit 25; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'], 'ms_per_step', d['ms_per_step'], 'fp32', r['fp32_values']['kernel_ms'])" "$OUT/r6_eab_$v$i.log" $v | tee -a "$OUT/r6_early_ab.txt"
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_band2.py tests/test_gpu_devbuild.py -q -x -s --timeout 600 --timeout-method thread > "$OUT/r6_early_tests.log" 2>&1 || { tail -40 "$OUT/r6_early_tests.log"; exit 23; }
grep -E "^build:|passed|failed" "$OUT/r6_early_tests.log" | tail -12
