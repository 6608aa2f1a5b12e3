#!/bin/bash
# A/B of bench.py invocations under rocprofv3 kernel stats.  CASES: ';'-separated
# "name|bench args" entries; each runs once (its own time limit), prints the bench line's
# head and the SpMV kernels' mean device time.  ENVS (optional, ';'-separated, same count):
# extra environment per case (e.g. SM_LIB_PATH=build/dev/libsparsematrix_amd.so SM_GCB_LOOK=42).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
IFS=';' read -ra CS <<< "$CASES"
IFS=';' read -ra EV <<< "${ENVS:-}"
for i in "${!CS[@]}"; do
  name=${CS[$i]%%|*}; args=${CS[$i]#*|}
  extra=${EV[$i]:-}
  extra=${extra//SM_LIB_PATH=build/SM_LIB_PATH=$ROOT/build}   # the run starts in /tmp
  rm -rf "$OUT/ab_$name"
  ( cd /tmp && env $extra timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ab_$name" -o run -- \
      python3 "$ROOT/bench.py" --no-cpu --no-spmm --no-rmat --no-config5 --no-fp32-values $args ) > "$OUT/ab_$name.log" 2>&1 || { tail -30 "$OUT/ab_$name.log"; exit 21; }
  echo "== $name ($extra) $args"; grep -h '^{' "$OUT/ab_$name.log" | tail -1 | cut -c1-200
  python3 - "$OUT/ab_$name" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "spmv" in n or "spmm" in n:
            print(f"  {float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>4}  {n[:100]}")
PY
done
echo r4_ab done
