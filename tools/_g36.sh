set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "comment" --timeout 200 --timeout-method thread > gpurun_out/g36_cmt.log 2>&1; rc=$?; tail -3 gpurun_out/g36_cmt.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g36_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/g36_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/g36_bench.log 2> gpurun_out/g36_bench.err || exit 1; python -c "
import json; d=json.loads(open('gpurun_out/g36_bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline'])"
