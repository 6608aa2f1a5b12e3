#!/bin/bash
# Per-rank SpMV kernel at emulated N-rank weak-scaling shapes (rank 0's 2^20 x N*2^20 slice
# on one GPU): rocprofv3 kernel stats per N through tools/r3_ab.sh.  VARIANTS as there
# (default: the in-tree library's AUTO).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for n in ${NS:-2 4 8}; do
  BENCH_ARGS="--emulate-world $n" VARIANTS="${VARIANTS:-auto=tree}" ROUNDS=1 bash tools/r3_ab.sh | sed "s/^/N=$n /" || exit 1
done
