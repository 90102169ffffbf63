#!/bin/bash
# Round evidence per bench config on the GPU box: the bench line (with the
# CPU baselines), rocprofv3 --kernel-trace --stats of the same bench, and the
# PMC passes (tools/gpu_pmc.sh: FETCH_SIZE, WRITE_SIZE, SQ).  usage:
#   TAG=r2 bash tools/r2_profile.sh libsvm_1m_x128 csv_1m_x256 ...
set -o pipefail
TAG=${TAG:-r2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for c in "$@"; do
  t=${TAG}_$c
  cd $R
  timeout -k 10 900 python bench.py --config $c --cpu-budget ${CPU_BUDGET:-10} > $O/bench_$t.json 2> $O/bench_$t.err || { tail -5 $O/bench_$t.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$t.json'));print('$c', d['value'], d['roofline']['avg_ms'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$t -o run -- \
    python3 $R/bench.py --config $c --no-cpu-baseline --steps 5 --warmup 1 > $O/rocprof_$t.log 2>&1 || { tail -5 $O/rocprof_$t.log; exit 1; }
  cd $R && BENCH_ARGS="--config $c" bash tools/gpu_pmc.sh $t > $O/pmc_$t.log 2>&1 || { tail -5 $O/pmc_$t.log; exit 1; }
  echo "$c profiled"
done
