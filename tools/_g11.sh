set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/g11_pytest.log 2>&1; rc=$?; tail -3 $O/g11_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --config libsvm_1m_x128 --no-cpu-baseline > $O/g11_bench.json 2> $O/g11_bench.err && python -c "import json;d=json.load(open('$O/g11_bench.json'));print(d['value'], d['roofline']['avg_ms'], d['roofline']['frac'])" && \
VARIANTS=base bash tools/ablate_pmc.sh
