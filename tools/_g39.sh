set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r2d bash tools/r2_profile.sh libsvm_1m_x128 libsvm_cmt_1m_x128 libsvm_qid_1m_x128 libfm_1m_x64
