set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/g5_pytest.log 2>&1; echo "pytest rc=$?"; grep -E "FAILED|Error|passed|failed" $O/g5_pytest.log | tail -15
timeout -k 10 300 python bench.py --config libsvm_1m_x128 --no-cpu-baseline > $O/g5_bench.json 2> $O/g5_bench.err && python -c "import json;d=json.load(open('$O/g5_bench.json'));print(d['value'], d['roofline']['avg_ms'], d['roofline']['frac'])"
