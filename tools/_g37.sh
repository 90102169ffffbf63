set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "comment_bench" --timeout 150 --timeout-method thread > gpurun_out/g37_t.log 2>&1; rc=$?; tail -2 gpurun_out/g37_t.log; [ $rc = 0 ] || exit $rc
TAG=r2c bash tools/r2_profile.sh libsvm_1m_x128 libsvm_cmt_1m_x128
