#!/bin/bash
# Round-6 end to end with the text DMA'd from registered page-cache mappings:
# host-API GPU tests, run_e2e (mapped, then DMLC_AMD_MMAP=0, then mapped
# again), and the host-only pipelines probe (pinned copy vs mapped) at 1 and 8
# pipelines.  usage: bash tools/gpu_r6_e2e.sh [tag]
set -o pipefail
TAG=${1:-r6_e2e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_host_api.py tests/test_plugin.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  && tail -1 $O/pytest.log \
  && DMLC_AMD_STATS=1 timeout -k 10 300 python tools/e2e/run_e2e.py > $O/e2e_mmap.jsonl 2> $O/e2e_mmap.err \
  && DMLC_AMD_MMAP=0 DMLC_AMD_STATS=1 timeout -k 10 300 python tools/e2e/run_e2e.py > $O/e2e_copy.jsonl 2> $O/e2e_copy.err \
  && DMLC_AMD_STATS=1 timeout -k 10 300 python tools/e2e/run_e2e.py > $O/e2e_mmap2.jsonl 2> $O/e2e_mmap2.err \
  && python3 -c "import sys; sys.path.insert(0,'.'); from tools import synth; t,_=synth.rows(synth.LIBSVM,1<<21,128,seed=1); open('/tmp/hp_libsvm.txt','wb').write(t.tobytes())" \
  && for P in 1 8; do for M in 0 1; do HOST_PIPES_MAPPED=$M DMLC_AMD_READ_THREADS=2 timeout -k 10 300 tools/e2e/_build/host_pipes /tmp/hp_libsvm.txt $P 3 32 0.55 2 >> $O/host_pipes.jsonl || exit 1; done; done \
  && cat $O/host_pipes.jsonl && echo e2e done
