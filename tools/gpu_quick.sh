#!/bin/bash
# Quick GPU iteration: selected parity tests (PYTEST_K filter), then the bench's SpMV
# under rocprofv3 kernel stats.  Every GPU step has its own limit; stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
if [[ -n "${PYTEST_K:-}" ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYTEST_K" > "$OUT/pytest_quick.log" 2>&1 || { tail -40 "$OUT/pytest_quick.log"; exit 11; }
  tail -2 "$OUT/pytest_quick.log"
fi
export TMPDIR=/tmp
rm -rf "$OUT/qprof"
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/qprof" -o run -- \
    python3 "$ROOT/bench.py" --steps 30 --warmup 5 --no-cpu --no-spmm --no-rmat ${BENCH_ARGS:-} ) > "$OUT/qprof.log" 2>&1 || { tail -30 "$OUT/qprof.log"; exit 14; }
grep -h '^{' "$OUT/qprof.log" | tail -1 | cut -c1-400
python3 - "$OUT/qprof" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "spmv" in n or "combine" in n:
            print(f"  {float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>4}  {n[:120]}")
PY
