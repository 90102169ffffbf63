#!/bin/bash
# GPU-box quick loop: parity suite + one bench line per config given (default libsvm).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_quick.log 2>&1
rc=$?
tail -3 $O/pytest_quick.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest_quick.log | head -20; exit $rc; }
for c in ${CONFIGS:-libsvm_1m_x128}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bq_$c.json 2> $O/bq_$c.err || { tail -5 $O/bq_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bq_$c.json'));print('$c', d['value'], 'GB/s', d['roofline']['avg_ms'], 'ms frac', d['roofline']['frac'], d['path'])"
done
