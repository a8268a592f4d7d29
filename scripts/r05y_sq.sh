# SQ counters of the final build's det and HUC-8 horizons (one pass each, 8 SQ counters)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
BENCH_ARGS="" bash scripts/gpu_pmc.sh r05y_detsq "$C" || exit $?
BENCH_ARGS="--huc8" bash scripts/gpu_pmc.sh r05y_huc8sq "$C" || exit $?
exit 0
