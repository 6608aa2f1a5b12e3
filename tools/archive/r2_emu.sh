set -o pipefail
cd $GRAFT_REPO_ROOT
for n in 4 8; do for lk in 3,2 5,2 6,3; do
  echo "N=$n GLOOK=$lk"; SM_XBAND_GLOOK=$lk BENCH_ARGS="--emulate-world $n" bash tools/r2_ab.sh || exit 1
done; done
