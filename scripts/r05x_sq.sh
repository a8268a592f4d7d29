# SQ wave-time breakdown (active / issue-stalled / parked) of the final build's det, ens64 and
# EnKF32 kernels: one pass each, 8 SQ counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"
BENCH_ARGS="" bash scripts/gpu_pmc.sh r05x_detsq "$C" || exit $?
BENCH_ARGS="--members 64" bash scripts/gpu_pmc.sh r05x_ens64sq "$C" || exit $?
BENCH_ARGS="--members 32 --enkf" bash scripts/gpu_pmc.sh r05x_enkf32sq "$C" || exit $?
exit 0
