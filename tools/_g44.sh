set -o pipefail
cd $GRAFT_REPO_ROOT
V=dmlc-core_amd/lib/variants
for lib in $V/pre.so dmlc-core_amd/lib/libdmlc_amd.so $V/noinl.so $V/pre.so dmlc-core_amd/lib/libdmlc_amd.so $V/noinl.so; do
DMLC_AMD_LIB=$lib timeout -k 10 200 python bench.py --config libsvm_1m_x128 --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/g44.log 2> gpurun_out/g44.err || exit 1; python -c "
import json; d=json.loads(open('gpurun_out/g44.log').read().strip().splitlines()[-1]); print('$lib'.split('/')[-1], d['roofline']['avg_ms'], d['ms_per_step'])"
done
DMLC_AMD_LIB=$V/noinl.so timeout -k 10 200 python bench.py --config libsvm_cmt_1m_x128 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/g44c.log 2> gpurun_out/g44.err || exit 1; tail -c 200 gpurun_out/g44c.log
