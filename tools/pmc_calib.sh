#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per access width (tools/ubench/pmc_calib.hip), one
# PMC counter per rocprofv3 run; summary: python tools/pmc_calib_read.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_calib; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/$c -o run -- $R/tools/_build/pmc_calib > $O/$c.log 2>&1 || exit 1
done
echo calib done
