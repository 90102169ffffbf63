set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python tools/stamps.py > $O/g25_stamps.log 2>&1; rc=$?; cat $O/g25_stamps.log; [ $rc = 0 ] || exit $rc
for c in libsvm_1m_x128 csv_1m_x256 libfm_1m_x64; do timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/g25_bench_$c.json 2> $O/g25_bench.err && python -c "import json;d=json.load(open('$O/g25_bench_$c.json'));print('$c', d['value'], d['path'], d['roofline']['avg_ms'], d['roofline']['frac'])" || exit 1; done
