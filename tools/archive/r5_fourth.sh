#!/bin/bash
# Round 5, fourth GPU session: two-buffer x-stream variants (xstream a), then the evidence
# passes (tools/r5_evidence.sh) and the instruction counts of gcb on R-MAT 24.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 120 ./build/xstream 50 a > "$OUT/r5_xstream_a.txt" 2>&1 || { tail -20 "$OUT/r5_xstream_a.txt"; exit 21; }
cat "$OUT/r5_xstream_a.txt"
bash tools/r5_evidence.sh || exit 22
export TMPDIR=/tmp
cd /tmp || exit 1
RMAT_GCB_NO_SHUFFLE=1 timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_rmat_gcb" -o run -- python3 "$ROOT/tools/rmat_gcb_ab.py" 24 0 > "$OUT/pmc_rmat_gcb.log" 2>&1 || { tail -20 "$OUT/pmc_rmat_gcb.log"; exit 23; }
tail -5 "$OUT/pmc_rmat_gcb.log"
