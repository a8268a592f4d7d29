#!/bin/bash
# Profiles of a build for profiles/: HBM traffic (det / ens64 / CONUS-16; FETCH_SIZE and
# WRITE_SIZE in separate passes, bench horizons only -> scripts/hbm_traffic.py on the host),
# kernel-trace stats (det / HUC-8 / ens64 / EnKF32 / EnKF256) and the SQ wave-time breakdown
# (det / ens64 / EnKF32 -> scripts/sq_breakdown.py).   Usage: bash scripts/round_profiles.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${1:-r06}"
O=gpurun_out
mkdir -p $O
BENCH_ARGS="" bash scripts/gpu_pmc.sh ${TAG}_det FETCH_SIZE WRITE_SIZE || exit $?
BENCH_ARGS="--members 64" bash scripts/gpu_pmc.sh ${TAG}_ens64 FETCH_SIZE WRITE_SIZE || exit $?
BENCH_ARGS="--conus" bash scripts/gpu_pmc.sh ${TAG}_conus FETCH_SIZE WRITE_SIZE || exit $?
stats() {   # name, bench args
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof_${TAG}_$name" \
      -o run -- python3 "$PWD/bench.py" --no-cpu --no-api --timing-runs 1 "$@" > $O/prof_${TAG}_$name.log 2>&1
  local rc=$?
  echo "stats $name rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $O/prof_${TAG}_$name.log; exit $rc; }
  return 0
}
stats det --steps 5 --warmup 1
stats huc8 --steps 5 --warmup 1 --huc8
stats ens64 --steps 2 --warmup 1 --members 64
stats enkf32 --steps 1 --warmup 1 --members 32 --enkf
stats enkf256 --steps 1 --warmup 1 --members 256 --enkf
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"
BENCH_ARGS="" bash scripts/gpu_pmc.sh ${TAG}_detsq "$C" || exit $?
BENCH_ARGS="--members 64" bash scripts/gpu_pmc.sh ${TAG}_ens64sq "$C" || exit $?
BENCH_ARGS="--members 32 --enkf" bash scripts/gpu_pmc.sh ${TAG}_enkf32sq "$C" || exit $?
exit 0
