set -o pipefail
cd $GRAFT_REPO_ROOT
for sd in 1 0; do HSA_ENABLE_SDMA=$sd timeout -k 10 400 python tools/e2e/run_e2e.py libsvm_1m_x128 csv_1m_x256 > gpurun_out/e2e_sdma$sd.jsonl 2> gpurun_out/e2e.err || exit 1; echo "sdma $sd"; python -c "
import json
for l in open('gpurun_out/e2e_sdma$sd.jsonl'):
    d=json.loads(l); print(d['config'], d['GBps'], d['best_s'], d['first_s'], d['stages_pass_s'], d['stages'])"; done
