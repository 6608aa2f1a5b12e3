set -o pipefail
cd $GRAFT_REPO_ROOT
RMAT_ABL=0 bash tools/r2_rmat.sh
