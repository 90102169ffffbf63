#!/bin/bash
# Round-6 final build on the GPU box: GPU parity suite, smoke, default bench
# line, 2-rank rehearsal over the one card, end to end (file -> Parser ->
# RowBlocks).  usage: bash tools/gpu_r6_final.sh [tag]
set -o pipefail
TAG=${1:-r6_final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  && tail -1 $O/pytest.log \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
  && timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && echo bench ok \
  && timeout -k 10 600 python bench.py --gpus 2 --no-cpu-baseline > $O/gpus2.json 2> $O/gpus2.err && echo gpus2 ok \
  && timeout -k 10 600 python tools/e2e/run_e2e.py > $O/e2e.jsonl 2> $O/e2e.err && echo e2e ok
