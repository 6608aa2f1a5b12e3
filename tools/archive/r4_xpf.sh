#!/bin/bash
# dma3 + XPF (band q+1's x and codebook values read during band q behind an LDS flag from the
# loader, dev_x1) vs the default: band tests on dev_x1, then a same-box A/B.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
SM_LIB_PATH=$ROOT/build/dev_x1/libsparsematrix_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_band2.py -q --timeout 200 --timeout-method thread > gpurun_out/r4_xpf_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_xpf_tests.log
[[ $rc -eq 0 ]] || exit $rc
D=SM_LIB_PATH=build/dev/libsparsematrix_amd.so
X=SM_LIB_PATH=build/dev_x1/libsparsematrix_amd.so
CASES="p0|--steps 30;p1|--steps 30;p0b|--steps 30;p1b|--steps 30;x0|--steps 30;x1|--steps 30" ENVS="$D;$X;$D;$X;$D SM_B2_XCDMAP=1;$X SM_B2_XCDMAP=1" bash tools/r4_ab.sh
