#!/bin/bash
# End-to-end engine knob sweep on the GPU box (copy mode x workers per device
# x batch bytes), libsvm config 2 by default: one JSON line per setting on stdout.
#   [MODES="kernel dma"] [WORKERS="2 3 4"] [BATCHES=...] [CONFIGS=...] bash tools/e2e_sweep.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
cd $R
export TMPDIR=${TMPDIR:-/tmp}
for m in ${MODES:-kernel}; do
for w in ${WORKERS:-2 3 4}; do
  for b in ${BATCHES:-33554432 67108864}; do
    t=${m}_w${w}_b${b}_p${PRECOPY:-1}
    DMLC_AMD_PRECOPY=${PRECOPY:-1} DMLC_AMD_COPY=$m DMLC_AMD_WORKERS=$w DMLC_AMD_BATCH_BYTES=$b timeout -k 10 300 python tools/e2e/run_e2e.py ${CONFIGS:-libsvm_1m_x128} > $O/e2e_$t.jsonl 2> $O/e2e_$t.err || { tail -3 $O/e2e_$t.err; exit 1; }
    python3 -c "
import json
for l in open('$O/e2e_$t.jsonl'):
    d=json.loads(l); print('copy $m workers $w batch $b precopy ${PRECOPY:-1}', d['config'], d.get('GBps'), d.get('stages'))"
  done
done
done
