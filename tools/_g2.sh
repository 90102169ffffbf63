set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/g9_pytest.log 2>&1; echo "pytest rc=$?"; tail -2 $O/g9_pytest.log
for c in libsvm_1m_x128 csv_1m_x256; do timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/g9_bench_$c.json 2> $O/g9_bench.err && python -c "import json;d=json.load(open('$O/g9_bench_$c.json'));print('$c', d['value'], d['roofline']['avg_ms'], d['roofline']['frac'])"; done
timeout -k 10 300 python tools/stamps.py > $O/g9_stamps.txt 2>&1; cat $O/g9_stamps.txt
