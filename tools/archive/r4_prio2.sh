#!/bin/bash
# dma3: applying waves at the default priority (SM_BAND2_PRIO=0) vs s_setprio 2, repeated.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
D=SM_LIB_PATH=build/dev/libsparsematrix_amd.so
CASES="a0|--steps 30;a2|--steps 30;b0|--steps 30;b2|--steps 30;c0|--steps 30;c2|--steps 30" ENVS="$D SM_BAND2_PRIO=0;$D;$D SM_BAND2_PRIO=0;$D;$D SM_BAND2_PRIO=0;$D" bash tools/r4_ab.sh
