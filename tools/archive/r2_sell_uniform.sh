set -o pipefail
cd $GRAFT_REPO_ROOT
SM_SELL=1 timeout -k 10 300 python3 tools/spmv_sweep.py --workload uniform --rows 1048576 --tiles 4096 --algos sell --replicas 4 --rounds 3 --reps 10 2>&1 | grep -v "^\[" | tail -4
SM_SELL=1 timeout -k 10 300 python3 tools/spmv_sweep.py --workload uniform --rows 131072 --per-row 16 --tiles 4096 --algos sell --replicas 4 --rounds 3 --reps 10 2>&1 | tail -3
