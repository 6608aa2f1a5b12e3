set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_sell.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sell.log 2>&1 || { tail -40 gpurun_out/pytest_sell.log; exit 11; }
tail -1 gpurun_out/pytest_sell.log
RMAT_ABL=0 bash tools/r2_rmat.sh | grep -v "^E20\|^W20"
