set -o pipefail
mkdir -p /tmp/csvt && printf '0,1,2,3\n4,5,6,7\n' > /tmp/csvt/part-00.txt && printf '8,9,10,11\n12,13,14,15' > /tmp/csvt/part-01.txt && printf '16,17,18,19\n' > /tmp/csvt/part-02.txt
for nt in 1 2; do DMLC_AMD_NTHREAD=$nt timeout 60 tests/cpp/_build/host_api_test /tmp/csvt 0 1 csv 32 f32 /tmp/o$nt; echo rc=$?; python -c "
import numpy as np
print('nt=$nt', np.fromfile('/tmp/o$nt.value',np.float32).tolist(), np.fromfile('/tmp/o$nt.offset',np.uint64).tolist(), np.fromfile('/tmp/o$nt.blocks',np.uint64).tolist())"; done
