set -o pipefail
cd $GRAFT_REPO_ROOT
V=dmlc-core_amd/lib/variants
for c in csv_1m_x256 libsvm_1m_x128; do for lib in $V/pre.so $V/head.so dmlc-core_amd/lib/libdmlc_amd.so $V/pre.so dmlc-core_amd/lib/libdmlc_amd.so; do
DMLC_AMD_LIB=$lib timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/g42.log 2> gpurun_out/g42.err || exit 1; python -c "
import json; d=json.loads(open('gpurun_out/g42.log').read().strip().splitlines()[-1]); print('$c', '$lib'.split('/')[-1], d['roofline']['avg_ms'], d['ms_per_step'])"
done; done
