#!/bin/bash
# A/B of SpMV builds and build options: rocprofv3 kernel stats of the config-2 bench per
# variant.  VARIANTS: space-separated name=lib[,VAR=value...]; lib "tree" is the in-tree
# library, otherwise build/<lib>/libsparsematrix_amd.so.  ROUNDS repeats the list.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for r in $(seq 1 "${ROUNDS:-2}"); do
for spec in $VARIANTS; do
  name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%,*}
  envs=(); [[ $rest == *,* ]] && IFS=',' read -ra envs <<< "${rest#*,}"
  if [[ $lib == tree ]]; then unset SM_LIB_PATH; else export SM_LIB_PATH=$GRAFT_REPO_ROOT/build/$lib/libsparsematrix_amd.so; fi
  rm -rf gpurun_out/ab/$name
  ( cd /tmp && env "${envs[@]}" timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab/$name -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-spmm --no-rmat --steps 30 --warmup 3 ${BENCH_ARGS:-} ) > gpurun_out/ab_$name.log 2>&1 || { echo "$name failed"; tail -20 gpurun_out/ab_$name.log; exit 1; }
  python3 - gpurun_out/ab/$name $name <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "spmv" in r["Name"]:
            print(f"{sys.argv[2]:14s} {float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
done
done
