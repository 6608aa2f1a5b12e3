#!/bin/bash
# Round 4 GPU check: selected -m gpu tests (PYTEST_K), the default bench (N = 1, with the
# config-5 and fp32-values sub-lines), and a 2-rank rehearsal of the N > 1 path on one GPU
# (bench.py launches its own ranks; the C-ABI context over a host-staged gloo all-gather).
# Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
STEPS=${STEPS:-tests,bench,rehearse}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/r4_tests.log" 2>&1 || { tail -60 "$OUT/r4_tests.log"; exit 11; }
  tail -3 "$OUT/r4_tests.log"
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > "$OUT/r4_bench.log" 2>&1 || { tail -30 "$OUT/r4_bench.log"; exit 12; }
  grep '^{' "$OUT/r4_bench.log" | tail -1 > "$OUT/r4_bench_line.json"
  cut -c1-600 "$OUT/r4_bench_line.json"
fi
if [[ $STEPS == *rehearse* ]]; then
  SM_BENCH_REHEARSE=1 timeout -k 10 600 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu --no-spmm --c5-global-rows $((1<<24)) > "$OUT/r4_rehearse.log" 2>&1 || { tail -30 "$OUT/r4_rehearse.log"; exit 13; }
  grep '^{' "$OUT/r4_rehearse.log" | tail -1 | cut -c1-1500
fi
echo r4_check done
