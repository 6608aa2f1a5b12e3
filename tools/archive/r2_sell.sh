# Sell-kernel check on one GPU: its GPU tests (+ the parity suite), the R-MAT scale-24
# column statistics and the R-MAT SpMV timing under rocprofv3 (tools/r2_rmat.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_sell.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ps.log 2>&1 || { tail -30 gpurun_out/ps.log; exit 11; }
tail -1 gpurun_out/ps.log
timeout -k 10 300 python3 tools/rmat_stats.py 2>&1 | tail -9
RMAT_ABL=0 bash tools/r2_rmat.sh | grep -v "^E20\|^W20" | grep "sell\|finalize\|relabel"
