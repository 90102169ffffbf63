set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_host_api.py -x -v --timeout 300 --timeout-method thread -k "config4 or config5 or max_index or multi_device" > $O/g13_pytest.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/g13_pytest.log | tail -12; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --config libsvm_qid_1m_x128 --steps 5 --warmup 1 --cpu-budget 8 > $O/g13_qid.json 2> $O/g13_qid.err; rc=$?; tail -c 1500 $O/g13_qid.json; tail -3 $O/g13_qid.err; exit $rc
