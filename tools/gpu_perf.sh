#!/bin/bash
# GPU-box perf iteration: parity tests, phase stamps, bench (no CPU baseline).
set -o pipefail
TAG=${1:-perf}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -2 $O/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/stamps.py > $O/stamps_$TAG.log 2>&1 && cat $O/stamps_$TAG.log \
  && timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS} > $O/bench_$TAG.json 2> $O/bench_$TAG.err \
  && cat $O/bench_$TAG.json
