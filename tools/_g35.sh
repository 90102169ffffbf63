set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g35_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/g35_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g35_smoke.log 2>&1 || exit 1; tail -1 gpurun_out/g35_smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/g35_bench.log 2> gpurun_out/g35_bench.err || exit 1; tail -c 1200 gpurun_out/g35_bench.log
