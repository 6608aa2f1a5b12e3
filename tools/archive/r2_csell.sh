#!/bin/bash
# Codebook sell (4-byte column|id words) vs the plain column + value form
# (SM_SELL_CB=0): sell GPU tests, then rocprofv3 kernel stats on R-MAT scale 24 and
# on the uniform config-2 shape without bands (development A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
[ -n "$NO_TESTS" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_sell.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/csell_tests.log 2>&1 || { tail -30 gpurun_out/csell_tests.log; exit 1; }
[ -n "$NO_TESTS" ] || tail -2 gpurun_out/csell_tests.log
for v in ${VARIANTS:-1:8 0:8}; do
  cb=${v%%:*}; un=${v#*:}
  for wl in rmat uniform; do
    if [ $wl = rmat ]; then a="--workload rmat --scale 24 --tiles 2048 --replicas 1 --reps 5"
    else a="--workload uniform --rows 1048576 --tiles 4096 --replicas 4 --reps 10"; fi
    d=$GRAFT_REPO_ROOT/gpurun_out/csell_${wl}_${cb}_$un
    rm -rf $d
    ( cd /tmp && SM_SELL=1 SM_XBAND=0 SM_SELL_CB=$cb SM_SELL_UNROLL=$un timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $d -o run -- python3 $GRAFT_REPO_ROOT/tools/spmv_sweep.py $a --algos sell --rounds 1 ) \
        > $d.log 2>&1 || { echo "$wl $v failed"; tail -20 $d.log; exit 1; }
    python3 - $d "$wl cb=$cb u=$un" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "sell" in r["Name"] or "relabel" in r["Name"] or "finalize" in r["Name"]:
            print(f"{sys.argv[2]:18s} {float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:60]}")
PY
  done
done
