set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "csv" --timeout 300 --timeout-method thread > gpurun_out/g41_csv.log 2>&1; rc=$?; tail -2 gpurun_out/g41_csv.log; [ $rc = 0 ] || exit $rc
for c in csv_1m_x256; do
timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/g41_$c.log 2> gpurun_out/g41_bench.err || exit 1; python -c "
import json; d=json.loads(open('gpurun_out/g41_$c.log').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['frac'], d.get('path'))"
done
timeout -k 10 300 python bench.py --config csv_1m_x256 --label-column 0 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/g41_lab.log 2> gpurun_out/g41_bench.err || exit 1; tail -c 300 gpurun_out/g41_lab.log
