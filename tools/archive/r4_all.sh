#!/bin/bash
# One GPU call, several steps (STEPS, comma-separated, in order): ab (tools/r4_ab.sh with
# CASES/ENVS), tests (pytest -m gpu, PYTEST_K filter), bench (default bench.py), rehearse
# (2 ranks on one GPU), c5 (config-5 layout A/B), rmat (R-MAT sell timeline, dev lib).
# Each step has its own time limit.  An ordinary failure (exit 1: a failed test or assert)
# moves on to the next step; a crash, abort or time limit (any other non-zero code) ends the
# call there.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
STEPS=${STEPS:-ab,tests,bench,rehearse}
worst=0
step() {   # name, command...
  local name=$1; shift
  echo "==== $name"
  "$@"
  local rc=$?
  echo "==== $name rc=$rc"
  if [[ $rc -ne 0 && $rc -ne 1 ]]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  [[ $rc -ne 0 ]] && worst=1
  return 0
}
run_tests() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/r4_tests.log" 2>&1
  local rc=$?
  tail -25 "$OUT/r4_tests.log"
  return $rc
}
run_bench() {
  timeout -k 10 700 python -u bench.py ${BENCH_ARGS:-} > "$OUT/r4_bench.log" 2>&1
  local rc=$?
  grep '^{' "$OUT/r4_bench.log" | tail -1 > "$OUT/r4_bench_line.json"
  cut -c1-800 "$OUT/r4_bench_line.json"; tail -3 "$OUT/r4_bench.log" | cut -c1-300
  [[ $rc -eq 0 ]] || return 1
}
run_rehearse() {
  SM_BENCH_REHEARSE=1 timeout -k 10 600 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu --no-spmm --c5-global-rows $((1<<24)) > "$OUT/r4_rehearse.log" 2>&1
  local rc=$?
  grep '^{' "$OUT/r4_rehearse.log" | tail -1 | cut -c1-1500; tail -3 "$OUT/r4_rehearse.log" | cut -c1-300
  [[ $rc -eq 0 ]] || return 1
}
run_rmat() {
  local rc
  for v in "ts|SM_SELL_TS=1" "nogather|SM_SELL_TS=1 SM_SELL_ABLATE=1"; do
    local nm=${v%%|*} ev=${v#*|}
    env SM_LIB_PATH=build/dev/libsparsematrix_amd.so $ev RMAT_PROF_REPS=2 timeout -k 10 300 python -u tools/rmat_prof.py > "$OUT/r4_rmat_$nm.log" 2>&1
    rc=$?
    echo "-- $nm ($ev)"; tail -16 "$OUT/r4_rmat_$nm.log"
    [[ $rc -eq 0 ]] || return $rc
  done
}
prof() {   # name, timeout, command...: rocprofv3 kernel stats of the command, summary printed
  local name=$1 lim=$2; shift 2
  rm -rf "$OUT/p_$name"
  ( cd /tmp && TMPDIR=/tmp timeout -k 10 "$lim" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p_$name" -o run -- "$@" ) > "$OUT/p_$name.log" 2>&1
  local rc=$?
  tail -12 "$OUT/p_$name.log" | cut -c1-300
  python3 - "$OUT/p_$name" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"  {float(r['AverageNs'])/1e3:9.2f} us  x{r['Calls']:>4}  {r['Name'][:110]}")
PY
  [[ $rc -eq 0 ]] || return $rc
}
run_sellpipe() {   # the sell tests on the dev library, pipelined loop off and on
  local rc=0
  for v in 0 1; do
    SM_LIB_PATH=$ROOT/build/dev/libsparsematrix_amd.so SM_SELL_PIPE=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_sell.py -q --timeout 120 --timeout-method thread > "$OUT/r4_sellpipe$v.log" 2>&1
    rc=$?
    echo "-- SM_SELL_PIPE=$v rc=$rc"; tail -4 "$OUT/r4_sellpipe$v.log"
    [[ $rc -eq 0 || $rc -eq 1 ]] || return $rc
  done
}
run_spmm() { prof spmm 300 python3 "$ROOT/tools/spmm_ab.py" --algos auto,mfma --n 32; }
run_native() { prof native 300 python3 "$ROOT/tools/native_bench.py"; }
run_nativeab() {   # m = 1: the counting-sort kernel (SM_NAT_SORT=1) vs the round-3 kernels (0), dev library
  local rc
  for v in 1 0 1 0; do
    SM_LIB_PATH=$ROOT/build/dev/libsparsematrix_amd.so SM_NAT_SORT=$v timeout -k 10 200 python3 tools/native_bench.py > "$OUT/r4_nat$v.log" 2>&1
    rc=$?
    echo "-- SM_NAT_SORT=$v"; grep -E "^(config1|16384)" "$OUT/r4_nat$v.log"
    [[ $rc -eq 0 ]] || return $rc
  done
}
run_blas() {
  SBLAS_REPS=9 timeout -k 10 300 ./build/blas_test 1:32 16384 16384 0 "sgemm_sparse;sm_addmatmat_auto" > "$OUT/r4_blas.log" 2>&1
  local rc=$?
  cat "$OUT/r4_blas.log" | head -20
  [[ $rc -eq 0 ]] || return $rc
}
IFS=',' read -ra ST <<< "$STEPS"
for s in "${ST[@]}"; do
  case $s in
    ab) step ab bash tools/r4_ab.sh ;;
    ab2) step ab2 env CASES="$CASES2" ENVS="${ENVS2:-}" bash tools/r4_ab.sh ;;
    tests) step tests run_tests ;;
    bench) step bench run_bench ;;
    rehearse) step rehearse run_rehearse ;;
    c5) step c5 bash tools/r4_c5.sh ;;
    rmat) step rmat run_rmat ;;
    spmm) step spmm run_spmm ;;
    sellpipe) step sellpipe run_sellpipe ;;
    native) step native run_native ;;
    nativeab) step nativeab run_nativeab ;;
    blas) step blas run_blas ;;
  esac
done
echo "r4_all done worst=$worst"
