# A/B of library builds under build/ab_*/ against the in-tree one (rocprofv3 kernel stats of bench.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in tree $(ls -d build/ab_* 2>/dev/null | xargs -n1 basename); do
  if [[ $v == tree ]]; then unset SM_LIB_PATH; else export SM_LIB_PATH=$GRAFT_REPO_ROOT/build/$v/libsparsematrix_amd.so; fi
  rm -rf gpurun_out/ab/$v
  ( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab/$v -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-spmm --no-rmat --steps 30 --warmup 3 ${BENCH_ARGS:-} ) > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -20 gpurun_out/ab_$v.log; exit 1; }
  python3 - gpurun_out/ab/$v $v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "spmv" in r["Name"]:
            print(f"{sys.argv[2]:12s} {float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
done
