# R-MAT scale 24 stream-kernel timing (rocprofv3 kernel stats), with and without the gather ablation
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for a in ${RMAT_ABL:-0 1}; do
  rm -rf gpurun_out/rmat$a
  ( cd /tmp && SM_STREAM_ABLATE=$a timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/rmat$a -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/spmv_sweep.py --workload rmat --scale 24 --tiles 2048 --algos "${RMAT_ALGOS:-sell}" --replicas 1 --rounds 1 --reps 5 ) > gpurun_out/rmat$a.log 2>&1 || { tail -20 gpurun_out/rmat$a.log; exit 1; }
  grep -h "stream" gpurun_out/rmat$a.log | tail -2
  python3 - gpurun_out/rmat$a <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "spmv" in r["Name"] or "sell" in r["Name"] or "relabel" in r["Name"] or "finalize" in r["Name"]:
            print(f"  {float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:100]}")
PY
done
