#!/bin/bash
# Full GPU parity suite, smoke and the default bench line on the GPU box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
cd $R
TAG=${TAG:-chk}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_$TAG.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/pytest_$TAG.log | tail -3
[ $rc = 0 ] || { grep -E "FAILED|Error" $O/pytest_$TAG.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 && tail -1 $O/smoke_$TAG.log || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$TAG.json 2> $O/bench_$TAG.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_$TAG.json'));print(d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['frac'], d['path'])"
