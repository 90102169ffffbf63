set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "comment or qid or fuzz" --timeout 200 --timeout-method thread > gpurun_out/g38_cmt.log 2>&1; rc=$?; tail -2 gpurun_out/g38_cmt.log; [ $rc = 0 ] || exit $rc
for c in libsvm_1m_x128 libsvm_cmt_1m_x128 libsvm_1m_x128; do
timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/g38_$c.log 2> gpurun_out/g38_bench.err || exit 1; python -c "
import json; d=json.loads(open('gpurun_out/g38_$c.log').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['frac'], d.get('path'))"
done
