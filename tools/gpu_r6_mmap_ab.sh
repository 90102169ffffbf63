#!/bin/bash
# A/B of the mapped text path's registration (segment size, portable flag)
# against the pinned copy, end to end on config 2.  usage: bash tools/gpu_r6_mmap_ab.sh [tag]
set -o pipefail
TAG=${1:-r6_mmap_ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
run() {  # name, env...
  local n=$1; shift
  env "$@" DMLC_AMD_STATS=1 timeout -k 10 300 python tools/e2e/run_e2e.py libsvm_1m_x128 > $O/$n.jsonl 2> $O/$n.err || return 1
  python3 -c "
import json
for l in open('$O/$n.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('$n', d['GBps'], d['GBps_stream'], d['best_s'], d['create_s'], d['delete_s'], d['stages']['read_s'], d['stages']['h2d_s'])"
}
run copy DMLC_AMD_MMAP=0 && run m64 DMLC_AMD_MMAP=1 && run m16 DMLC_AMD_MMAP=1 DMLC_AMD_MMAP_SEG_MB=16 \
  && run m256 DMLC_AMD_MMAP=1 DMLC_AMD_MMAP_SEG_MB=256 && run m64p DMLC_AMD_MMAP=1 DMLC_AMD_MMAP_PORTABLE=1 \
  && run copy2 DMLC_AMD_MMAP=0 && run m64b DMLC_AMD_MMAP=1
