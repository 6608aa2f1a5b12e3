#!/bin/bash
# dma3 tall vs dma3: tile timelines (SM_BAND2_ABLATE=2048, dev build) and the no-hand-off /
# no-apply ablations of dma3 tall (rocprofv3 means).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
mkdir -p gpurun_out
DEV=$ROOT/build/dev/libsparsematrix_amd.so
for bt in 4 7; do
  SM_LIB_PATH=$DEV SM_BAND2_ABLATE=2048 timeout -k 10 300 python -u tools/cband_prof.py band_tall=$bt \
    > gpurun_out/r4_tl_$bt.log 2>&1 || { tail -20 gpurun_out/r4_tl_$bt.log; exit 3; }
  echo "== timeline band_tall=$bt"; grep -A4 "tile timeline" gpurun_out/r4_tl_$bt.log | tail -5; head -1 gpurun_out/r4_tl_$bt.log
done
D=SM_LIB_PATH=build/dev/libsparsematrix_amd.so
CASES="t|--steps 30 --band-tall 7;t_nohand|--steps 30 --band-tall 7;t_noapply|--steps 30 --band-tall 7;d_nohand|--steps 30" \
ENVS="$D;$D SM_BAND2_ABLATE=8;$D SM_BAND2_ABLATE=1;$D SM_BAND2_ABLATE=8" bash tools/r4_ab.sh
