set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r3a NO_CPU= bash tools/profile_configs.sh libsvm_1m_x128 csv_1m_x256 || exit 1
TAG=r3a NO_PMC=1 NO_CPU=1 bash tools/profile_configs.sh libsvm_im1_1m_x128 csv_i32_1m_x256 csv_sp_1m_x256 || exit 1
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python bench.py --gpus 2 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r3a_gpus2.json 2> gpurun_out/r3a_gpus2.err; echo "gpus2 rc=$?"; tail -2 gpurun_out/r3a_gpus2.err; cat gpurun_out/r3a_gpus2.json
