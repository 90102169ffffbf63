set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/g23_pytest.log 2>&1; rc=$?; tail -3 $O/g23_pytest.log; [ $rc = 0 ] || exit $rc
for c in libfm_1m_x64 libsvm_1m_x128 libsvm_qid_1m_x128; do timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/g23_bench_$c.json 2> $O/g23_bench.err && python -c "import json;d=json.load(open('$O/g23_bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['frac'])" || exit 1; done
