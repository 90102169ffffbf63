set -o pipefail
VARIANTS="base kb3 kb5 prio" bash tools/ab.sh || exit 1
VARIANTS="base kb3 prio" BENCH_ARGS="--config libfm_1m_x64" bash tools/ab.sh || exit 1
