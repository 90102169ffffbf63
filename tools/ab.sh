#!/bin/bash
# A/B: bench each variant library (lib/variants/*.so) interleaved, 2 passes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd $R
for pass in 1 2; do
  for v in ${VARIANTS:-$(ls dmlc-core_amd/lib/variants/ | sed 's/.so$//')}; do
    DMLC_AMD_LIB=$R/dmlc-core_amd/lib/variants/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 ${BENCH_ARGS} > $O/ab_$v.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$O/ab_$v.json'));print('$v pass $pass', d['value'], d['roofline']['avg_ms'], d['path'])"
  done
done
