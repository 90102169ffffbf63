set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python tools/e2e/run_e2e.py libsvm_1m_x128 csv_1m_x256 > gpurun_out/r2d_e2e.jsonl 2> gpurun_out/e2e.err || { tail -5 gpurun_out/e2e.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r2d_e2e.jsonl'):
    d=json.loads(l); print(d['config'], d['GBps'], d['best_s'], d['first_s'], d['stages_pass_s'], d['stages'], d.get('cpu_reference'))"
