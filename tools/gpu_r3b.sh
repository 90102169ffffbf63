set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=base bash tools/pmc_diag.sh
