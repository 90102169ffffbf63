set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g45_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/g45_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g45_smoke.log 2>&1 || exit 1; tail -1 gpurun_out/g45_smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/g45_bench.log 2> gpurun_out/g45_bench.err || exit 1; python -c "
import json; d=json.loads(open('gpurun_out/g45_bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])"
