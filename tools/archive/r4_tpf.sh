#!/bin/bash
# dma3: codebook values read a band early (SM_LD_TPF=1, default) vs with the band (dev_t0).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_band2.py -q --timeout 200 --timeout-method thread > gpurun_out/r4_tpf_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_tpf_tests.log
[[ $rc -eq 0 ]] || exit $rc
D=SM_LIB_PATH=build/dev/libsparsematrix_amd.so
T=SM_LIB_PATH=build/dev_t0/libsparsematrix_amd.so
CASES="on|--steps 30;off|--steps 30;on2|--steps 30;off2|--steps 30" ENVS="$D;$T;$D;$T" bash tools/r4_ab.sh
