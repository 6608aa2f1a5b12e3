#!/bin/bash
# Config 5 rank-0-of-8 slice: gather-band kind vs gathered chunk bands (gcb), rocprofv3
# kernel stats of each (bench.py --workload config5 --emulate-world 8 --layout ...).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
for L in ${LAYOUTS:-gcb gather}; do
  rm -rf "$OUT/c5_$L"
  ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5_$L" -o run -- \
      python3 "$ROOT/bench.py" --workload config5 --emulate-world 8 --steps 10 --warmup 2 --replays 3 --no-cpu --layout $L ) > "$OUT/c5_$L.log" 2>&1 || { tail -30 "$OUT/c5_$L.log"; exit 21; }
  echo "== $L"; grep -h '^{' "$OUT/c5_$L.log" | tail -1 | cut -c1-300
  python3 - "$OUT/c5_$L" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "spmv" in n:
            print(f"  {float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>4}  {n[:110]}")
PY
done
echo r4_c5 done
