#!/bin/bash
# Device time of a kernel's ablation variants (development only): for each value V
# in $VARIANTS, run the bench under rocprofv3 --kernel-trace --stats with
# $ABL_ENV=V and print the per-kernel average durations of the SpMV kernels.
#   ABL_ENV=SM_CTILE_ABLATE VARIANTS="0 1 2 4 8" bash tools/ablate.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/ablate
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
for v in ${VARIANTS:-0}; do
  export "${ABL_ENV:-SM_CTILE_ABLATE}=$v"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/v$v" -o run -- \
      python3 "$ROOT/bench.py" --no-cpu --no-spmm --no-rmat --steps 20 --warmup 3 ${BENCH_ARGS:-} > "$OUT/v$v.log" 2>&1 \
      || { echo "variant $v failed"; tail -20 "$OUT/v$v.log"; exit 1; }
  echo "== variant $v"
  python3 - "$OUT/v$v" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "spmv" in n or "combine" in n:
            print(f"  {float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>4}  {n[:110]}")
PY
done
