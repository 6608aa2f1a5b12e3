#!/bin/bash
# Round 3 GPU session: the default bench (config 2 + SpMM + R-MAT + CPU baselines),
# config 5's rank-0 slice at 8 ranks (emulated on one GPU), and a 2-rank rehearsal of
# the N > 1 bookkeeping (both ranks on GPU 0, gloo data path).  Stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
STEPS=${STEPS:-bench,config5,rehearse}
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 13; }
  grep '^{' "$OUT/bench.log" | tail -1 | cut -c1-600
fi
if [[ $STEPS == *config5* ]]; then
  timeout -k 10 900 python -u bench.py --workload config5 --emulate-world ${EMU:-8} --steps 20 --warmup 3 --no-cpu ${C5_ARGS:-} > "$OUT/config5_emu.log" 2>&1 || { tail -30 "$OUT/config5_emu.log"; exit 15; }
  grep '^{' "$OUT/config5_emu.log" | tail -1 | cut -c1-600
fi
if [[ $STEPS == *rehearse* ]]; then
  SM_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu --no-spmm --no-rmat > "$OUT/rehearse2.log" 2>&1 || { tail -30 "$OUT/rehearse2.log"; exit 16; }
  grep '^{' "$OUT/rehearse2.log" | tail -1 | cut -c1-600
fi
echo "r3_bench done"
