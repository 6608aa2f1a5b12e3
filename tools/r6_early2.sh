#!/bin/bash
# Round 6: where the early publish's loop time goes -- tile timelines of dev_n (no early publish),
# dev_x1 (the code present, never run), dev_x2 (the loader's LDS reads, no stores), dev_e (full).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
lib() { echo "$ROOT/build/dev_$1/libsparsematrix_amd.so"; }
for v in n x1 x2 e; do
  SM_LIB_PATH=$(lib $v) SM_BAND2_PROF=2 timeout -k 10 150 python -u tools/cband_prof.py > "$OUT/r6_tl5_$v.txt" 2>&1 || { tail -20 "$OUT/r6_tl5_$v.txt"; exit 22; }
  echo "== $v"; grep -v "^  tile" "$OUT/r6_tl5_$v.txt" | tail -n 9 | head -4
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_devbuild.py -q -x -s --timeout 600 --timeout-method thread > "$OUT/r6_devbuild_tests.log" 2>&1 || { tail -40 "$OUT/r6_devbuild_tests.log"; exit 23; }
grep -E "^build:|passed|failed" "$OUT/r6_devbuild_tests.log" | tail -12
