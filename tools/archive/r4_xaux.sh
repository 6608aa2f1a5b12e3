#!/bin/bash
# gcb: cache-policy bits of the x gathers (SM_GCB_XAUX: 0 default, 1 sc0, 2 nt, 16 sc1, 17 sc0 sc1),
# config 5 rank-0 slice, rocprofv3 kernel stats (dev build).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
D=SM_LIB_PATH=build/dev/libsparsematrix_amd.so
A="--workload config5 --emulate-world 8 --steps 10 --replays 3 --layout gcb"
CASES="a0|$A;a1|$A;a2|$A;a16|$A;a17|$A" ENVS="$D SM_GCB_XAUX=0;$D SM_GCB_XAUX=1;$D SM_GCB_XAUX=2;$D SM_GCB_XAUX=16;$D SM_GCB_XAUX=17" bash tools/r4_ab.sh
# R-MAT 24 codebook sell with the same policies (tools/rmat_ab.py: median of 20 SpMVs)
for a in -1 16 2 17 1; do
  echo "-- SM_SELL_XAUX=$a"
  SM_LIB_PATH=$ROOT/build/dev/libsparsematrix_amd.so SM_SELL_XAUX=$a timeout -k 10 300 python3 tools/rmat_ab.py 24 "{}" 2>&1 | tail -2 || exit 41
done
