#!/bin/bash
# Round 6, first GPU session: the cband tile timeline with the hand-off's phases stamped,
# for the round-5 hand-off (build/dev_a: SM_B2_BL=0) and the beta-last one (build/dev_b);
# alternating A/B of the bench's config-2 line; the band tests and a full bench line on the
# product build.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
for v in a b; do
  SM_B2_TS_DUMP=1 SM_LIB_PATH=$ROOT/build/dev_$v/libsparsematrix_amd.so SM_BAND2_PROF=2 \
    timeout -k 10 150 python -u tools/cband_prof.py > "$OUT/r6_tl_$v.txt" 2>&1 || { tail -20 "$OUT/r6_tl_$v.txt"; exit 21; }
  grep -v "^  tile" "$OUT/r6_tl_$v.txt" | tail -n 9
done
: > "$OUT/r6_bl_ab.txt"
for i in 1 2 3; do
  for v in a b; do
    SM_LIB_PATH=$ROOT/build/dev_$v/libsparsematrix_amd.so timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 \
      --no-cpu --no-spmm --no-rmat --no-config5 > "$OUT/r6_ab_$v$i.log" 2>&1 || { tail -20 "$OUT/r6_ab_$v$i.log"; exit 22; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'], 'ms_per_step', d['ms_per_step'], 'fp32', r['fp32_values']['kernel_ms'])" "$OUT/r6_ab_$v$i.log" $v | tee -a "$OUT/r6_bl_ab.txt"
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_band2.py -q -x --timeout 300 --timeout-method thread > "$OUT/r6_band2_tests.log" 2>&1 || { tail -40 "$OUT/r6_band2_tests.log"; exit 23; }
tail -n 2 "$OUT/r6_band2_tests.log"
timeout -k 10 600 python -u bench.py > "$OUT/r6_bench_full.log" 2>&1 || { tail -20 "$OUT/r6_bench_full.log"; exit 24; }
tail -n 1 "$OUT/r6_bench_full.log" > "$OUT/r6_bench_line.json"
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); r=d['roofline']; print('full bench: kernel_ms', r['kernel_ms'], 'ms_per_step', d['ms_per_step'], 'fp32', r['fp32_values']['kernel_ms'], 'again', r.get('replay_after_legs_ms'))" "$OUT/r6_bench_line.json"
