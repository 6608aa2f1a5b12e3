#!/bin/bash
# dma3 tall (band_tall = 7): its band tests, then config 2 A/B against the default dma3.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_band2.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4_tall_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4_tall_tests.log; echo "tests rc=$rc"; [[ $rc -eq 0 ]] || exit $rc
CASES="d|--steps 30;t|--steps 30 --band-tall 7;d2|--steps 30;t2|--steps 30 --band-tall 7" bash tools/r4_ab.sh
