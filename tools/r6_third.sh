#!/bin/bash
# Round 6, third GPU session: publish ablations of the beta-last hand-off (SM_B2_ABL, timeline
# only): p1 plain stores, p2 plain stores + agent release/acquire (a valid form: checked bit for
# bit, then A/B against write-through), p3 a quarter of the rows.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
lib() { echo "$ROOT/build/dev_$1/libsparsematrix_amd.so"; }
for v in b p1 p2 p3; do
  SM_B2_TS_DUMP=1 SM_LIB_PATH=$(lib $v) SM_BAND2_PROF=2 timeout -k 10 150 python -u tools/cband_prof.py > "$OUT/r6_tl3_$v.txt" 2>&1 || { tail -20 "$OUT/r6_tl3_$v.txt"; exit 21; }
  echo "== $v"; grep -v "^  tile" "$OUT/r6_tl3_$v.txt" | tail -n 9
done
SM_LIB_PATH=$(lib p2) timeout -k 10 300 python -u tools/handoff_check.py > "$OUT/r6_check_p2.txt" 2>&1 || { tail -20 "$OUT/r6_check_p2.txt"; exit 22; }
cat "$OUT/r6_check_p2.txt"
: > "$OUT/r6_pub_ab.txt"
for i in 1 2 3; do
  for v in b p2; do
    SM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 \
      --no-cpu --no-spmm --no-rmat --no-config5 > "$OUT/r6_pab_$v$i.log" 2>&1 || { tail -20 "$OUT/r6_pab_$v$i.log"; exit 25; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'], 'ms_per_step', d['ms_per_step'], 'fp32', r['fp32_values']['kernel_ms'])" "$OUT/r6_pab_$v$i.log" $v | tee -a "$OUT/r6_pub_ab.txt"
  done
done
