#!/bin/bash
# Profiles of the frozen build for the round: HBM traffic (FETCH_SIZE / WRITE_SIZE, one counter
# per pass) of the det, ens64 and CONUS-16 bench workloads, kernel-trace stats of the det /
# ens64 / EnKF32 / EnKF256 workloads, and the smoke.  Usage: bash scripts/final_profiles.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${1:-r04}"
O=gpurun_out
mkdir -p $O
BENCH_ARGS="" bash scripts/gpu_pmc.sh ${TAG}_det FETCH_SIZE WRITE_SIZE || exit $?
BENCH_ARGS="--members 64" bash scripts/gpu_pmc.sh ${TAG}_ens64 FETCH_SIZE WRITE_SIZE || exit $?
BENCH_ARGS="--conus" bash scripts/gpu_pmc.sh ${TAG}_conus FETCH_SIZE WRITE_SIZE || exit $?
stats() {   # name, bench args
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof_$name" \
      -o run -- python3 "$PWD/bench.py" --no-cpu --no-api --timing-runs 1 "$@" > $O/prof_$name.log 2>&1
  local rc=$?
  echo "stats $name rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $O/prof_$name.log; exit $rc; }
  return 0
}
stats det --steps 5 --warmup 1
stats ens64 --steps 2 --warmup 1 --members 64
stats enkf32 --steps 2 --warmup 1 --members 32 --enkf
stats enkf256 --steps 1 --warmup 1 --members 256 --enkf
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"
exit $rc
