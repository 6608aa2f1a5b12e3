#!/bin/bash
# Slab combine: no load for the own slab's part (default) vs the round-3 form (dev_c0).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
D=SM_LIB_PATH=build/dev/libsparsematrix_amd.so
C=SM_LIB_PATH=build/dev_c0/libsparsematrix_amd.so
CASES="s1|--steps 30;s0|--steps 30;s1b|--steps 30;s0b|--steps 30" ENVS="$D;$C;$D;$C" bash tools/r4_ab.sh
