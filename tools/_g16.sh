set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/g16_pytest.log 2>&1; rc=$?; tail -3 $O/g16_pytest.log; [ $rc = 0 ] || exit $rc
for c in libsvm_qid_1m_x128 libsvm_1m_x128; do timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/g16_bench_$c.json 2> $O/g16_bench.err && python -c "import json;d=json.load(open('$O/g16_bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['frac'])" || exit 1; done
R=$(pwd); cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_g16 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/$O/g16_prof.log 2>&1 && cut -c1-160 $R/$O/prof_g16/run_kernel_stats.csv | head -8
