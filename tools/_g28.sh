set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "libsvm or libfm or config or fuzz or qid or csv" --timeout 300 --timeout-method thread > $O/g28_pytest.log 2>&1; rc=$?; tail -3 $O/g28_pytest.log; [ $rc = 0 ] || exit $rc
VARIANTS="head lb lbl32" bash tools/ab.sh || exit 1
VARIANTS="head lb lbl32" BENCH_ARGS="--config csv_1m_x256" bash tools/ab.sh || exit 1
VARIANTS="head lb" BENCH_ARGS="--config libfm_1m_x64" bash tools/ab.sh || exit 1
