#!/bin/bash
# Round evidence on the GPU box: bench (with CPU baseline), rocprofv3
# --kernel-trace --stats of the same bench command, and PMC passes.
set -o pipefail
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python bench.py ${BENCH_ARGS} > $O/bench_$TAG.json 2> $O/bench_$TAG.err && cat $O/bench_$TAG.json || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- \
  python3 $R/bench.py --no-cpu-baseline ${BENCH_ARGS} > $O/rocprof_$TAG.log 2>&1 || exit 1
cd $R && bash tools/gpu_pmc.sh $TAG > /dev/null && echo pmc ok
