set -o pipefail
TAG=r2b CPU_BUDGET=10 bash tools/r2_profile.sh libsvm_1m_x128 csv_1m_x256 libfm_1m_x64
