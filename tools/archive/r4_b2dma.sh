#!/bin/bash
# band2 (8-byte entries) in the dma3 geometry: band tests, then the fp32-values sub-line's
# kernel with the default (wide) vs SM_BAND_TALL=4 (dma3), rocprofv3 stats, dev build.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_band2.py -q --timeout 200 --timeout-method thread > gpurun_out/r4_b2dma_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_b2dma_tests.log
[[ $rc -eq 0 ]] || exit $rc
export TMPDIR=/tmp
for v in "w|" "d|SM_BAND_TALL=4" "w2|" "d2|SM_BAND_TALL=4" "c0|SM_LIB_PATH=$ROOT/build/dev_c0/libsparsematrix_amd.so" "c1|" ; do
  nm=${v%%|*}; ev=${v#*|}
  rm -rf gpurun_out/b2d_$nm
  ( cd /tmp && env SM_LIB_PATH=$ROOT/build/dev/libsparsematrix_amd.so $ev timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/b2d_$nm -o run -- \
      python3 $ROOT/bench.py --no-cpu --no-spmm --no-rmat --no-config5 --steps 30 ) > gpurun_out/b2d_$nm.log 2>&1 || { tail -20 gpurun_out/b2d_$nm.log; exit 21; }
  echo "== $nm ($ev)"
  python3 - gpurun_out/b2d_$nm <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "band2" in r["Name"]:
            print(f"  {float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
done
