#!/bin/bash
# gcb column pacing: correctness (gcb tests on the dev library with SM_GCB_PACE) and an A/B
# of the slack on config 5's rank-0 slice, then the PMC traffic passes of the default.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT" || exit 1
SM_LIB_PATH=$ROOT/build/dev/libsparsematrix_amd.so SM_GCB_PACE=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_gcb.py -q --timeout 200 --timeout-method thread > gpurun_out/r4_pace_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_pace_tests.log
[[ $rc -eq 0 ]] || exit $rc
D=SM_LIB_PATH=build/dev/libsparsematrix_amd.so
A="--workload config5 --emulate-world 8 --steps 10 --replays 3 --layout gcb"
CASES="p0|$A;p2|$A;p4|$A;p8|$A;p1|$A" ENVS="$D;$D SM_GCB_PACE=2;$D SM_GCB_PACE=4;$D SM_GCB_PACE=8;$D SM_GCB_PACE=1" bash tools/r4_ab.sh || exit $?
[[ -n "${NO_PMC:-}" ]] || PMC_CMD="python3 $ROOT/bench.py --workload config5 --emulate-world 8 --steps 5 --warmup 1 --replays 1 --no-cpu --layout gcb" bash tools/pmc.sh > gpurun_out/pmc_c5.txt 2>&1
tail -2 gpurun_out/pmc_c5.txt
