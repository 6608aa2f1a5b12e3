#!/bin/bash
# dma3 cband geometry: its GPU tests, then a same-box A/B against the default (wide) cband
# on config 2 (rocprofv3 kernel stats, two alternating runs each).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_band2.py -q -k "dma3" --timeout 200 --timeout-method thread > "$OUT/r4_dma3_tests.log" 2>&1
rc=$?
tail -5 "$OUT/r4_dma3_tests.log"
[[ $rc -eq 0 ]] || exit $rc
CASES="w0|--steps 30;d0|--steps 30 --band-tall 4;w1|--steps 30;d1|--steps 30 --band-tall 4" bash tools/r4_ab.sh
