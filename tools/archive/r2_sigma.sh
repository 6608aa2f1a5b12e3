#!/bin/bash
# R-MAT scale 24, sell path: sort windows (SM_SELL_SIGMA rows) and XCD streams
# (SM_SELL_STREAMS) A/B, rocprofv3 kernel stats per variant (development only).
#   VARIANTS="0:1 65536:8 65536:1" bash tools/r2_sigma.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in ${VARIANTS:-0:1 16384:8 65536:8 262144:8 65536:1}; do
  sig=${v%%:*}; st=${v#*:}
  rm -rf gpurun_out/sig_$sig_$st
  ( cd /tmp && SM_SELL_SIGMA=$sig SM_SELL_STREAMS=$st timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $GRAFT_REPO_ROOT/gpurun_out/sig_${sig}_$st -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/spmv_sweep.py --workload rmat --scale 24 --tiles 2048 --algos sell --replicas 1 --rounds 1 --reps 5 ) \
      > gpurun_out/sig_${sig}_$st.log 2>&1 || { echo "variant $v failed"; tail -20 gpurun_out/sig_${sig}_$st.log; exit 1; }
  python3 - gpurun_out/sig_${sig}_$st "sigma=$sig streams=$st" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "sell" in r["Name"] or "relabel" in r["Name"] or "finalize" in r["Name"]:
            print(f"{sys.argv[2]:28s} {float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:70]}")
PY
done
