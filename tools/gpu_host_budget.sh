#!/bin/bash
# Host-side evidence for the end-to-end pipeline on the GPU box (VERDICT r4
# items 5 and 8): the link probe's copy-size sweep and batched pipeline shapes,
# host memcpy, and P concurrent host pipelines without GPU work
# (tools/e2e/host_pipes).  Outputs gpurun_out/host_<tag>.jsonl.
set -o pipefail
TAG=${1:-r5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
J=$O/host_$TAG.jsonl
cd $R
python3 -c "
import json, os
q = open('/sys/fs/cgroup/cpu.max').read().split() if os.path.exists('/sys/fs/cgroup/cpu.max') else ['?']
cpu = [l.split(':',1)[1].strip() for l in open('/proc/cpuinfo') if l.startswith('model name')]
mem = [l for l in open('/proc/meminfo') if l.startswith('MemTotal')][0].split()[1]
print(json.dumps({'case': 'host', 'cpu': cpu[0] if cpu else '?', 'nproc_visible': os.cpu_count(),
                  'affinity': len(os.sched_getaffinity(0)), 'cgroup_cpu_max': ' '.join(q), 'mem_kib': int(mem)}))" > $J
timeout -k 10 300 python3 tools/e2e/link_probe.py 0 sweep batched >> $J || exit 1
echo "link probe done"
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, '.')
from tools import synth
t, _ = synth.rows(synth.LIBSVM, 2 << 20, 128, seed=1)
open('/tmp/hp.svm', 'wb').write(t.tobytes())" || exit 1
for P in 1 2 4 8; do
  timeout -k 10 120 tools/e2e/_build/host_pipes /tmp/hp.svm $P 3 32 0.5 4 >> $J || exit 1
done
for P in 8; do
  DMLC_AMD_READ_THREADS=2 timeout -k 10 120 tools/e2e/_build/host_pipes /tmp/hp.svm $P 3 32 0.5 1 >> $J || exit 1
done
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, 'tools/e2e'); sys.argv = ['x']
import link_probe; link_probe.host_memcpy(threads=(1, 4, 8, 16, 32))" >> $J || exit 1
rm -f /tmp/hp.svm
cat $J | wc -l
