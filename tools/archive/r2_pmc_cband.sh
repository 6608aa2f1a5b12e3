# PMC traffic + SQ/LDS counters of the bench's AUTO SpMV kernel (one rocprofv3 pass per group)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/pmc.sh > gpurun_out/pmc.txt 2>&1 || { tail -20 gpurun_out/pmc.txt; exit 2; }
python3 tools/pmc_traffic.py gpurun_out/pmc spmv_band2 spmv_1048576x1048576_16_per_row cband 150994948 > gpurun_out/traffic_cband.json 2>&1 || exit 3
PMC_CMD="python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu --no-spmm --no-rmat" bash tools/pmc_kernel.sh > gpurun_out/pmck.txt 2>&1 || { tail -20 gpurun_out/pmck.txt; exit 4; }
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu ) > gpurun_out/prof.log 2>&1 || exit 5
cat gpurun_out/traffic_cband.json; grep -A30 "band2_kernel<0" gpurun_out/pmck.txt
