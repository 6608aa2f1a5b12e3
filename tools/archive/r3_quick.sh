#!/bin/bash
# Quick GPU iteration: selected -m gpu tests (PYTEST_K), then selected bench lines.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
if [[ -n "${PYTEST_K:-}" ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > "$OUT/pytest_quick.log" 2>&1 || { tail -40 "$OUT/pytest_quick.log"; exit 11; }
  tail -2 "$OUT/pytest_quick.log"
fi
if [[ -n "${BENCH1:-}" ]]; then
  timeout -k 10 900 python -u bench.py $BENCH1 > "$OUT/bench1.log" 2>&1 || { tail -30 "$OUT/bench1.log"; exit 13; }
  grep '^{' "$OUT/bench1.log" | tail -1 | cut -c1-900
fi
if [[ -n "${BENCH2:-}" ]]; then
  timeout -k 10 900 python -u bench.py $BENCH2 > "$OUT/bench2.log" 2>&1 || { tail -30 "$OUT/bench2.log"; exit 14; }
  grep '^{' "$OUT/bench2.log" | tail -1 | cut -c1-900
fi
echo "r3_quick done"
