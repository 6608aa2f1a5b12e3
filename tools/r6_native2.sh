#!/bin/bash
# Round 6: the decode forms of the two-kernel native path -- 0 bitmap (per batch and group), 2 counting sort per batch (the product default);
# form 1 (a counting sort per batch and group, 29.2 us) was removed after this A/B:
# the native GPU tests on the product library, a same-box A/B of the development build
# (SM_NAT_DECODE, alternating), per-workgroup stamps of form 2 (SM_NAT_TS), and
# kernel-trace stats of 16384^2 at 0.1 %, m = 1.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread "$ROOT/tests/test_gpu_parity.py" -k "native or addmatmat" \
  > "$OUT/r6n2_tests.txt" 2>&1 || { tail -30 "$OUT/r6n2_tests.txt"; exit 20; }
tail -3 "$OUT/r6n2_tests.txt"
: > "$OUT/r6n2_ab.txt"
for v in 0 2 0 2; do
  echo "SM_NAT_DECODE=$v" >> "$OUT/r6n2_ab.txt"
  SM_LIB_PATH=$ROOT/build/dev/libsparsematrix_amd.so SM_NAT_DECODE=$v NATIVE_ALGOS=native \
    timeout -k 10 200 python3 "$ROOT/tools/native_bench.py" >> "$OUT/r6n2_ab.txt" 2>&1 || { tail -20 "$OUT/r6n2_ab.txt"; exit 21; }
done
cat "$OUT/r6n2_ab.txt"
SM_LIB_PATH=$ROOT/build/dev/libsparsematrix_amd.so SM_NAT_TS=1 NATIVE_CASES=16384 NATIVE_M=1 NATIVE_ALGOS=native \
  timeout -k 10 200 python3 "$ROOT/tools/native_bench.py" 2>&1 | grep "ts (us" | tail -3 > "$OUT/r6n2_ts.txt" || { echo ts failed; exit 23; }
cat "$OUT/r6n2_ts.txt"
rm -rf "$OUT/n2stat"
( cd /tmp && NATIVE_CASES=16384 NATIVE_M=1 NATIVE_ALGOS=native timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/n2stat" -o run -- python3 "$ROOT/tools/native_bench.py" ) > "$OUT/n2stat.log" 2>&1 || { tail -20 "$OUT/n2stat.log"; exit 22; }
find "$OUT/n2stat" -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-200
