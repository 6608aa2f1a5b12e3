#!/bin/bash
# Round 3 measurement session: PMC HBM traffic and SQ/LDS/TA/TD counters of config 2's AUTO
# kernel (cband), the rocprofv3 kernel stats of the default bench, and config 5 at p = 1
# (the whole 2^26 x 2^26 matrix on one GPU), and rocprofv3 kernel stats of tools/native_bench.py.  Each GPU step has its own time limit; the
# chain stops at the first failure.  STEPS selects: pmc, stats, c5p1, natprof.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
STEPS=${STEPS:-pmc,stats,c5p1,natprof}
if [[ $STEPS == *pmc* ]]; then
  bash tools/pmc.sh > "$OUT/pmc.txt" 2>&1 || { tail -20 "$OUT/pmc.txt"; exit 21; }
  python3 tools/pmc_traffic.py "$OUT/pmc" spmv_band2 spmv_1048576x1048576_16_per_row cband 150994948 > "$OUT/traffic_cband.json" 2>&1 || exit 22
  PMC_CMD="python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu --no-spmm --no-rmat" bash tools/pmc_kernel.sh > "$OUT/pmck.txt" 2>&1 || { tail -20 "$OUT/pmck.txt"; exit 23; }
  cat "$OUT/traffic_cband.json"
fi
if [[ $STEPS == *stats* ]]; then
  export TMPDIR=/tmp
  rm -rf "$OUT/prof"
  ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu ) > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 24; }
  grep '^{' "$OUT/prof.log" | tail -1 | cut -c1-300
fi
if [[ $STEPS == *c5p1* ]]; then
  timeout -k 10 900 python -u bench.py --workload config5 --steps 10 --warmup 2 --replays 1 --no-cpu > "$OUT/config5_p1.log" 2>&1 || { tail -30 "$OUT/config5_p1.log"; exit 25; }
  grep '^{' "$OUT/config5_p1.log" | tail -1 | cut -c1-600
fi
if [[ $STEPS == *natprof* ]]; then
  export TMPDIR=/tmp
  rm -rf "$OUT/natprof"
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/natprof" -o run -- python3 "$ROOT/tools/native_bench.py" ) > "$OUT/natprof.log" 2>&1 || { tail -20 "$OUT/natprof.log"; exit 26; }
fi
echo "r3_measure done"
