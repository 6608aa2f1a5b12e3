#!/bin/bash
# Emulated 2-rank slice (development only): blocked kind with and without LDS-DMA x staging,
# and the band2 kind forced, under tools/r2_ab.sh.
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 1 0; do echo "DMA=$v"; SM_XBAND_DMA=$v BENCH_ARGS="--emulate-world 2" bash tools/r2_ab.sh | grep tree; done
echo "band2 forced"; SM_XBAND_KIND=band2 BENCH_ARGS="--emulate-world 2" bash tools/r2_ab.sh | grep tree
