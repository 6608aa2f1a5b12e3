#!/bin/bash
# TA/TD/SQ counters over tools/ta_bench.hip (calibration of per-instruction costs).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmcta
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
G1="TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"
G2="SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
i=0
for g in "$G1" "$G2"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $g --kernel-trace --output-format csv -d "$OUT/g$i" -o run -- "$ROOT/build/ta_bench" > "$OUT/g$i.log" 2>&1 || { tail -20 "$OUT/g$i.log"; exit 31; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, os
from collections import defaultdict
root = sys.argv[1]
rows = defaultdict(dict)
order = []
for path in sorted(glob.glob(os.path.join(root, "g*", "**", "*counter_collection.csv"), recursive=True)):
    per = defaultdict(lambda: defaultdict(float)); names = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"]); names[d] = r["Kernel_Name"]
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    for j, d in enumerate(sorted(per)):
        key = j
        if key not in order: order.append(key)
        rows[key]["name"] = names[d][:40]
        rows[key].update(per[d])
for k in order:
    r = rows[k]
    print(k, r.pop("name"), " ".join(f"{c}={v:.0f}" for c, v in sorted(r.items())))
PY
