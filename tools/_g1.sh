set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/g1_pytest.log 2>&1; echo "pytest rc=$?"; tail -2 $O/g1_pytest.log
timeout -k 10 300 python bench.py --config libsvm_1m_x128 --no-cpu-baseline > $O/g1_bench.json 2> $O/g1_bench.err && cat $O/g1_bench.json | head -c 1500
echo; timeout -k 10 300 python tools/stamps.py > $O/g1_stamps.txt 2>&1; cat $O/g1_stamps.txt
