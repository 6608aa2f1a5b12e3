#!/bin/bash
# dma3 ablations (dev build, results wrong): no band barriers (512), no hand-off (8), both (520),
# no apply (1) -- the upper bound a barrier-free band loop could reach.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
D=SM_LIB_PATH=build/dev/libsparsematrix_amd.so
CASES="full|--steps 30;nobar|--steps 30;nohand|--steps 30;nobar_nohand|--steps 30;noapply|--steps 30;full_b|--steps 30;nobar_b|--steps 30" ENVS="$D;$D SM_BAND2_ABLATE=512;$D SM_BAND2_ABLATE=8;$D SM_BAND2_ABLATE=520;$D SM_BAND2_ABLATE=1;$D;$D SM_BAND2_ABLATE=512" bash tools/r4_ab.sh
