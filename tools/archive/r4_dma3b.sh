#!/bin/bash
# dma3 tuning A/B on config 2: default dma3 (loader prio 3), loader prio 0, entries 3 bands
# ahead, 7168-column windows with 8 table copies; wide cband as the reference point.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_band2.py -q -k "dma3" --timeout 200 --timeout-method thread > gpurun_out/r4_dma3_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_dma3_tests.log
[[ $rc -eq 0 ]] || exit $rc
D=SM_LIB_PATH=build/dev/libsparsematrix_amd.so
CASES="w|--steps 30;d|--steps 30 --band-tall 4;dp0|--steps 30 --band-tall 4;de3|--steps 30 --band-tall 4;dt|--steps 30 --band-tall 5;w2|--steps 30;d2|--steps 30 --band-tall 4;dp02|--steps 30 --band-tall 4;de32|--steps 30 --band-tall 4;dt2|--steps 30 --band-tall 5" \
ENVS="$D;$D;SM_LIB_PATH=build/dev_p0/libsparsematrix_amd.so;SM_LIB_PATH=build/dev_e3/libsparsematrix_amd.so;$D;$D;$D;SM_LIB_PATH=build/dev_p0/libsparsematrix_amd.so;SM_LIB_PATH=build/dev_e3/libsparsematrix_amd.so;$D" \
bash tools/r4_ab.sh
