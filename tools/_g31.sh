set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "api or plugin or split or cache" --timeout 300 --timeout-method thread > gpurun_out/g31_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/g31_pytest.log; [ $rc = 0 ] || exit $rc
for rt in 8 16; do DMLC_AMD_READ_THREADS=$rt timeout -k 10 400 python tools/e2e/run_e2e.py libsvm_1m_x128 csv_1m_x256 > gpurun_out/e2e_rt$rt.jsonl 2> gpurun_out/e2e.err || exit 1; echo "read threads $rt"; python -c "
import json
for l in open('gpurun_out/e2e_rt$rt.jsonl'):
    d=json.loads(l); print(d['config'], d['GBps'], d['best_s'], d['first_s'], d['stages_pass_s'], d['stages'])"; done
