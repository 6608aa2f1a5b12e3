#!/bin/bash
# MFMA counters of config 3's SpMM kernels (bench.py's spmm line and its mfma_variant): one
# rocprofv3 PMC pass with --kernel-trace only; the per-dispatch averages of every kernel
# whose name contains one of $KERNELS (default: spmm_rowpanel2 spmm_mfma) go to
# gpurun_out/mfma_<kernel>.json (copied to profiles/ by hand).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_mfma
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
CTR="SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d "$OUT/g1" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --replays 1 --no-cpu --no-rmat --no-config5 --no-fp32-values > "$OUT/g1.log" 2>&1 || { tail -20 "$OUT/g1.log"; exit 31; }
python3 - "$OUT" "$ROOT/gpurun_out" ${KERNELS:-spmm_rowpanel2 spmm_mfma} <<'PY'
import csv, glob, json, sys
from collections import defaultdict
csv.field_size_limit(1 << 30)
per = defaultdict(lambda: defaultdict(float)); names = {}
for path in glob.glob(sys.argv[1] + "/g1/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(path)):
        d = row["Dispatch_Id"]; names[d] = row["Kernel_Name"]
        c = row["Counter_Name"]
        v = float(row["Counter_Value"])
        per[d][c] = max(per[d][c], v) if c == "GRBM_GUI_ACTIVE" else per[d][c] + v
for sub in sys.argv[3:]:
    sel = [d for d in per if sub in names[d]]
    if not sel:
        print("no dispatch of", sub); continue
    avg = {c: sum(per[d][c] for d in sel) / len(sel) for c in per[sel[0]]}
    simds = 256 * 4
    util = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] * simds) if avg["GRBM_GUI_ACTIVE"] else None
    out = {"kernel": names[sel[0]][:160], "dispatches": len(sel), "counters_avg": avg,
           "mfma_util": util, "mfma_insts": avg.get("SQ_INSTS_VALU_MFMA_F32", 0) + avg.get("SQ_INSTS_MFMA", 0),
           "formula": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 1024 SIMDs) (rocprofv3 MfmaUtil, gfx94x derived formula)"}
    json.dump(out, open(f"{sys.argv[2]}/mfma_{sub}.json", "w"), indent=1)
    print(json.dumps(out)[:700])
PY
