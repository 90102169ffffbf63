#!/bin/bash
# Round-end evidence on the GPU box: parity suite, smoke, the default bench line
# (CPU baseline + HBM copy context), CSV and configs 4/5 bench lines, rocprof
# kernel stats of the default bench.  usage: bash tools/round_final.sh <tag>
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$TAG.log 2>&1 \
  && tail -1 $O/pytest_$TAG.log \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 && tail -1 $O/smoke_$TAG.log \
  && timeout -k 10 600 python bench.py > $O/bench_${TAG}_libsvm.json 2> $O/bench_${TAG}_libsvm.err && echo libsvm ok \
  && timeout -k 10 600 python bench.py --config csv_1m_x256 > $O/bench_${TAG}_csv.json 2> $O/bench_${TAG}_csv.err && echo csv ok \
  && timeout -k 10 600 python bench.py --config libsvm_32m_x64 --no-cpu-baseline > $O/bench_${TAG}_cfg5.json 2> $O/bench_${TAG}_cfg5.err && echo cfg5 ok \
  && timeout -k 10 900 python bench.py --config libsvm_1m_x2048 --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_${TAG}_cfg4.json 2> $O/bench_${TAG}_cfg4.err && echo cfg4 ok \
  && cd /tmp && export TMPDIR=/tmp \
  && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline > $O/rocprof_$TAG.log 2>&1 \
  && echo rocprof ok
