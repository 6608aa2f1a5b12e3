#!/bin/bash
# Round 6, second GPU session: correctness of the beta-last and combiner-tile hand-offs
# (tools/handoff_check.py, bit for bit), then tile timelines and an alternating A/B of the bench's
# config-2 line: a = round-5 hand-off (SM_B2_BL=0), b = beta-last, cNNNN = combiner tiles with
# the combiner slab at NNNN permille (SM_B2_COMB).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
B=$ROOT/build/dev_b/libsparsematrix_amd.so
SM_LIB_PATH=$B timeout -k 10 300 python -u tools/handoff_check.py > "$OUT/r6_check_b.txt" 2>&1 || { tail -20 "$OUT/r6_check_b.txt"; exit 21; }
cat "$OUT/r6_check_b.txt"
SM_B2_COMB=1120 SM_LIB_PATH=$B timeout -k 10 300 python -u tools/handoff_check.py > "$OUT/r6_check_c.txt" 2>&1 || { tail -20 "$OUT/r6_check_c.txt"; exit 22; }
cat "$OUT/r6_check_c.txt"
run_tl() {   # name lib [comb]
  SM_B2_COMB=${3:-0} SM_B2_TS_DUMP=1 SM_LIB_PATH=$2 SM_BAND2_PROF=2 timeout -k 10 150 python -u tools/cband_prof.py > "$OUT/r6_tl2_$1.txt" 2>&1 || { tail -20 "$OUT/r6_tl2_$1.txt"; exit 23; }
  echo "== $1"; grep -v "^  tile" "$OUT/r6_tl2_$1.txt" | tail -n 9
}
run_tl a "$ROOT/build/dev_a/libsparsematrix_amd.so" && run_tl b "$B" && run_tl c1000 "$B" 1000 && run_tl c1120 "$B" 1120 && run_tl c1200 "$B" 1200 || exit 24
: > "$OUT/r6_comb_ab.txt"
for i in 1 2; do
  for v in a b c1060 c1120 c1180; do
    case $v in a) L=$ROOT/build/dev_a/libsparsematrix_amd.so; C=0;; b) L=$B; C=0;; c*) L=$B; C=${v#c};; esac
    SM_B2_COMB=$C SM_LIB_PATH=$L timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 \
      --no-cpu --no-spmm --no-rmat --no-config5 > "$OUT/r6_cab_$v$i.log" 2>&1 || { tail -20 "$OUT/r6_cab_$v$i.log"; exit 25; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'], 'ms_per_step', d['ms_per_step'], 'fp32', r['fp32_values']['kernel_ms'])" "$OUT/r6_cab_$v$i.log" $v | tee -a "$OUT/r6_comb_ab.txt"
  done
done
