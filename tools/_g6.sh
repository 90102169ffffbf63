set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_host_api.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/g6_pytest.log 2>&1; echo "pytest rc=$?"; grep -E "FAILED|Error|passed|failed" $O/g6_pytest.log | tail -15
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
