#!/bin/bash
# dma3 with the slab tiles of a row block on one XCD (SM_B2_XCDMAP=1) vs default placement.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
D=SM_LIB_PATH=build/dev/libsparsematrix_amd.so
CASES="x0|--steps 30;x1|--steps 30;x0b|--steps 30;x1b|--steps 30" ENVS="$D;$D SM_B2_XCDMAP=1;$D;$D SM_B2_XCDMAP=1" bash tools/r4_ab.sh
