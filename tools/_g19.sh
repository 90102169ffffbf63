set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python tools/e2e/run_e2e.py libsvm_1m_x128 csv_1m_x256 > gpurun_out/r2_e2e.jsonl 2> gpurun_out/r2_e2e.err || exit 1
cat gpurun_out/r2_e2e.jsonl | cut -c1-200
TAG=r2 CPU_BUDGET=10 bash tools/r2_profile.sh libsvm_32m_x64 || exit 1
