#!/bin/bash
# dma3 builder A/B: cross-chunk bank balancing of single terms (default) vs off (SM_B2_BAL=0).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_band2.py tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread > gpurun_out/r4_bal_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_bal_tests.log
[[ $rc -eq 0 ]] || exit $rc
D=SM_LIB_PATH=build/dev/libsparsematrix_amd.so
CASES="on|--steps 30;off|--steps 30;on2|--steps 30;off2|--steps 30" ENVS="$D;$D SM_B2_BAL=0;$D;$D SM_B2_BAL=0" bash tools/r4_ab.sh
