#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 run, as
# MI355X_MICROARCH.md's rocprofv3 section prescribes); outputs under gpurun_out/pmc_<tag>/.
set -o pipefail
TAG=${1:-pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$name -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $O/$name.log 2>&1
}
run fetch FETCH_SIZE && run write WRITE_SIZE || exit 1
[ -n "$PMC_TRAFFIC_ONLY" ] && { echo pmc done; exit 0; }
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES \
  && run sq2 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  && ls $O/*/ && echo pmc done
