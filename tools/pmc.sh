#!/bin/bash
# rocprofv3 PMC passes for the HBM traffic of the bench's SpMV kernel, one counter
# group per run (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950), each
# with --kernel-trace only, plus the same passes over the calibration microbench
# (a 1 GiB float4 stream read of known size).  Output: gpurun_out/pmc/<name>/...
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=${PMC_OUT:-$ROOT/gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
BENCH=${PMC_CMD:-"python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu --no-spmm --no-rmat ${BENCH_ARGS:-}"}
for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo "$ctr" | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/bench_$tag" -o run -- $BENCH > "$OUT/bench_$tag.log" 2>&1 || { tail -20 "$OUT/bench_$tag.log"; exit 21; }
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/micro_$tag" -o run -- "$ROOT/build/microbench" > "$OUT/micro_$tag.log" 2>&1 || { tail -20 "$OUT/micro_$tag.log"; exit 22; }
done
echo "pmc done"
