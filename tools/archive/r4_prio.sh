#!/bin/bash
# dma3: the applying waves' s_setprio during the apply (SM_BAND2_PRIO 0..3, default 2), dev build.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
D=SM_LIB_PATH=build/dev/libsparsematrix_amd.so
CASES="q2|--steps 30;q0|--steps 30;q1|--steps 30;q3|--steps 30;q2b|--steps 30;q3b|--steps 30" ENVS="$D;$D SM_BAND2_PRIO=0;$D SM_BAND2_PRIO=1;$D SM_BAND2_PRIO=3;$D;$D SM_BAND2_PRIO=3" bash tools/r4_ab.sh
