#!/bin/bash
# Round-6 record run: the GPU test suite, the default bench line, rocprofv3 kernel stats of
# the bench's config-2 run, the PMC traffic passes (tools/pmc.sh) and the 2-rank rehearsal of
# the N > 1 bookkeeping (SM_BENCH_REHEARSE, both ranks on GPU 0).  Stops at the first
# crash / time limit.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
STEPS=${STEPS:-tests,bench,stats,pmc,rehearse}
if [[ ,$STEPS, == *,tests,* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/r6f_tests.log" 2>&1
  rc=$?; tail -4 "$OUT/r6f_tests.log"; echo "tests rc=$rc"
  [[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
fi
if [[ ,$STEPS, == *,smoke,* || $STEPS == *tests* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/r6f_smoke.log" 2>&1 || { tail -20 "$OUT/r6f_smoke.log"; exit 30; }
  tail -1 "$OUT/r6f_smoke.log"
fi
if [[ ,$STEPS, == *,bench,* ]]; then
  timeout -k 10 700 python -u bench.py > "$OUT/r6f_bench.log" 2>&1 || { tail -20 "$OUT/r6f_bench.log"; exit 31; }
  grep '^{' "$OUT/r6f_bench.log" | tail -1 > "$OUT/r6f_bench_line.json"; cut -c1-600 "$OUT/r6f_bench_line.json"
fi
if [[ ,$STEPS, == *,stats,* ]]; then
  rm -rf "$OUT/r6f_stats"
  ( cd /tmp && TMPDIR=/tmp timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r6f_stats" -o run -- \
      python3 "$ROOT/bench.py" --no-cpu --no-config5 --no-fp32-values ) > "$OUT/r6f_stats.log" 2>&1 || { tail -20 "$OUT/r6f_stats.log"; exit 32; }
  grep -h '^{' "$OUT/r6f_stats.log" | tail -1 > "$OUT/r6f_stats_line.json"
  echo "stats done"
fi
if [[ ,$STEPS, == *,pmc,* ]]; then
  BENCH_ARGS="--no-config5 --no-fp32-values" bash tools/pmc.sh || exit $?
fi
if [[ ,$STEPS, == *,rehearse,* ]]; then
  SM_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu --no-spmm --no-rmat > "$OUT/r6f_rehearse.log" 2>&1 || { tail -20 "$OUT/r6f_rehearse.log"; exit 33; }
  grep '^{' "$OUT/r6f_rehearse.log" | tail -1 > "$OUT/r6f_rehearse_line.json"; cut -c1-300 "$OUT/r6f_rehearse_line.json"
fi
echo "r6_final done"
