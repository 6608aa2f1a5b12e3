#!/bin/bash
# Round 5: the MFMA SpMM with its gathered X rows staged through LDS (spmm_mfma_lds_kernel):
# the MFMA tests on the release build (LDS form by default), then the register / LDS A/B on
# config 3 through the development build (SM_SPMM_MFMA_LDS=1 "old" = LDS, 0 "new" = registers).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_spmm_mfma.py -q -x --timeout 240 --timeout-method thread > "$OUT/r5_spmm_lds_tests.log" 2>&1 || { tail -30 "$OUT/r5_spmm_lds_tests.log"; exit 20; }
tail -1 "$OUT/r5_spmm_lds_tests.log"
: > "$OUT/r5_spmm_lds_ab.txt"
for rep in 1 2; do
  SM_LIB_PATH=$ROOT/build/dev/libsparsematrix_amd.so timeout -k 10 200 python -u tools/spmm_ab.py --ab-env SM_SPMM_MFMA_LDS --algo mfma --reps 50 >> "$OUT/r5_spmm_lds_ab.txt" 2>&1 || { tail -20 "$OUT/r5_spmm_lds_ab.txt"; exit 21; }
done
grep ab_env "$OUT/r5_spmm_lds_ab.txt"
rm -rf "$OUT/spmm_lds_stats"
( cd /tmp && TMPDIR=/tmp timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/spmm_lds_stats" -o run -- \
    python3 "$ROOT/tools/spmm_ab.py" --algos auto,mfma --reps 50 ) > "$OUT/spmm_lds_stats.log" 2>&1 || { tail -20 "$OUT/spmm_lds_stats.log"; exit 22; }
find "$OUT/spmm_lds_stats" -name '*kernel_stats.csv' -exec grep -h "spmm" {} \; | cut -c1-60,200-320
