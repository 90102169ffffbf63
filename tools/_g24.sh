set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "csv or config3 or plugin or api" --timeout 300 --timeout-method thread > $O/g24_pytest.log 2>&1; rc=$?; tail -4 $O/g24_pytest.log; [ $rc = 0 ] || exit $rc
for c in csv_1m_x256; do timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/g24_bench_$c.json 2> $O/g24_bench.err && python -c "import json;d=json.load(open('$O/g24_bench_$c.json'));print('$c', d['value'], d['path'], d['roofline']['avg_ms'], d['roofline']['frac'])" || exit 1; done
