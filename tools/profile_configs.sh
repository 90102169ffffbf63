#!/bin/bash
# Round evidence per bench config on the GPU box.  The bench line is the
# output of the profiled run itself: rocprofv3 --kernel-trace --stats wraps
# `bench.py --config <c>`, so profiles/<tag>_<c>_kernel_stats.csv and the line
# come from the same launches.  Then the PMC passes (tools/gpu_pmc.sh:
# FETCH_SIZE, WRITE_SIZE, SQ) unless NO_PMC=1.
#   TAG=r3 [NO_PMC=1] [NO_CPU=1] bash tools/profile_configs.sh libsvm_1m_x128 csv_1m_x256 ...
# Summarise afterwards (in the container): python tools/summarize_prof.py gpurun_out <tag>_<c> [kernel]
set -o pipefail
TAG=${TAG:-r3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for c in "$@"; do
  t=${TAG}_$c
  extra=""
  [ -n "$NO_CPU" ] && extra="--no-cpu-baseline"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$t -o run -- \
    python3 $R/bench.py --config $c --cpu-budget ${CPU_BUDGET:-10} $extra ${BENCH_EXTRA} > $O/bench_$t.out 2> $O/bench_$t.err \
    || { tail -5 $O/bench_$t.err; exit 1; }
  grep '^{' $O/bench_$t.out | tail -1 > $O/bench_$t.json
  python3 -c "import json;d=json.load(open('$O/bench_$t.json'));print('$c', d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['frac'], d['path'], (d.get('cpu_baseline') or {}).get('value'))"
  if [ -z "$NO_PMC" ]; then
    cd $R && BENCH_ARGS="--config $c ${BENCH_EXTRA}" bash tools/gpu_pmc.sh $t > $O/pmc_$t.log 2>&1 || { tail -5 $O/pmc_$t.log; exit 1; }
  fi
  echo "$c profiled"
done
