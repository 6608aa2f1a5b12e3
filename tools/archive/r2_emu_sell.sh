#!/bin/bash
# Per-rank slice at N ranks (bench.py --emulate-world N): AUTO (band kinds) vs the
# codebook sell (SM_XBAND=0), rocprofv3 kernel stats (development A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT
for n in ${NS:-2 4 8}; do
  for xb in 1 0; do
    echo "N=$n SM_XBAND=$xb"
    SM_XBAND=$xb BENCH_ARGS="--emulate-world $n" bash tools/r2_ab.sh || exit 1
  done
done
