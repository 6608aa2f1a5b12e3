#!/bin/bash
# Round 6: the merge-path session (tools/r6_merge.sh), then the reference-format decode's tests
# and counters (tools/r6_native.sh).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
bash tools/r6_merge.sh || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x -k "native or golden or addmatmat" --timeout 300 --timeout-method thread > gpurun_out/r6_native_tests.log 2>&1 || { tail -30 gpurun_out/r6_native_tests.log; exit 40; }
tail -n 1 gpurun_out/r6_native_tests.log
bash tools/r6_native.sh || exit $?
