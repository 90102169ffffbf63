set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "3 33554432" "2 67108864" "4 16777216"; do set -- $cfg; DMLC_AMD_WORKERS=$1 DMLC_AMD_BATCH_BYTES=$2 timeout -k 10 400 python tools/e2e/run_e2e.py libsvm_1m_x128 csv_1m_x256 > gpurun_out/e2e_w$1_b$2.jsonl 2> gpurun_out/e2e.err || exit 1; echo "workers $1 batch $2"; python -c "
import json
for l in open('gpurun_out/e2e_w$1_b$2.jsonl'):
    d=json.loads(l); print(d['config'], d['GBps'], d['best_s'], d['first_s'], d['stages_pass_s'], d['stages'])"; done
