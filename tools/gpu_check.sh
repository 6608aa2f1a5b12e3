#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench and a rocprofv3 kernel
# trace of the bench.  Every GPU step has its own time limit; the chain stops at
# the first failure.  Outputs land in gpurun_out/ (copied back by gpurun).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
STEPS=${STEPS:-all}
run() { echo "== $*" ; "$@"; }
if [[ $STEPS == all || $STEPS == *tests* ]]; then
  run timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 11; }
  tail -3 "$OUT/pytest_gpu.log"
fi
if [[ $STEPS == all || $STEPS == *smoke* ]]; then
  run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 12; }
  tail -1 "$OUT/smoke.log"
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
  run timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 13; }
  tail -1 "$OUT/bench.log"
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  rm -rf "$OUT/prof"
  ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu ) > "$OUT/prof.log" 2>&1 || { tail -30 "$OUT/prof.log"; exit 14; }
  find "$OUT/prof" -name '*stats*' | head
fi
echo "gpu_check done"
