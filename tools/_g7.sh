set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_plugin.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/g7_pytest.log 2>&1; echo "pytest rc=$?"; grep -E "FAILED|Error|passed|failed|assert" $O/g7_pytest.log | tail -15
