#!/bin/bash
# GPU-box check: parity tests, smoke, bench, rocprof kernel trace.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh [tag]
set -o pipefail
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1 \
  && tail -3 $O/pytest_gpu_$TAG.log \
  && echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 \
  && cat $O/smoke_$TAG.log \
  && echo "== bench" && timeout -k 10 600 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err \
  && cat $O/bench_$TAG.json \
  && echo "== rocprof" && cd /tmp && export TMPDIR=/tmp \
  && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/rocprof_$TAG.log 2>&1 \
  && find $O/prof_$TAG -name '*stats*' | head -5
