#!/bin/bash
# Multi-epoch end to end (one Parser, BeforeFirst between epochs): the pinned
# copy against the mapped text with its registrations kept across epochs.
#   bash tools/gpu_r6_epochs.sh [tag]
set -o pipefail
TAG=${1:-r6_epochs}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
python3 -c "import sys; sys.path.insert(0,'.'); from tools import synth; t,_=synth.rows(synth.LIBSVM,1<<20,128,seed=1); open('/tmp/ep_libsvm.txt','wb').write(t.tobytes()); t,_=synth.rows(synth.CSV,1<<20,256,seed=1); open('/tmp/ep_csv.txt','wb').write(t.tobytes())" || exit 1
for rep in 1 2; do for f in libsvm csv; do for m in 0 1; do
  DMLC_AMD_MMAP=$m timeout -k 10 300 tools/e2e/_build/e2e_bench /tmp/ep_$f.txt $f 1 5 2>> $O/err.txt | grep epochs | sed "s/^{/{\"mmap\": $m, /" | tee -a $O/epochs.jsonl || exit 1
done; done; done
