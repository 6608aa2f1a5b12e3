#!/bin/bash
# GPU tests (all), then the x-gather cache-policy A/B (tools/r4_xaux.sh), then the default
# bench line with rocprofv3 kernel stats.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4n_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4n_tests.log; echo "tests rc=$rc"
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
bash tools/r4_xaux.sh || exit $?
STEPS=stats bash tools/r4_final.sh
