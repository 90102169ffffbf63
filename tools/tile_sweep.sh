#!/bin/bash
# Exact-kernel tile-size sweep (tools/time_variant.py with TILE_BYTES) on the
# GPU box: FMT=exact|csv_exact [SIZES="131072 262144 ..."] bash tools/tile_sweep.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for t in ${SIZES:-131072 262144 524288 1048576}; do
  TILE_BYTES=$t timeout -k 10 120 python tools/time_variant.py ${FMT:-exact} || exit 1
done
