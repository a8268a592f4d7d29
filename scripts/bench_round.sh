#!/bin/bash
# Bench lines of the round (with CPU baselines): det (the default bench), ens64, EnKF32, EnKF256
# CONUS-16 (configs[4], one GPU's shard) and the full-covariance KF.  Usage: bash scripts/bench_round.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="${1:-r01}"
O=gpurun_out
mkdir -p $O
run() {   # name, command...
  local name=$1; shift
  timeout -k 10 300 "$@" > $O/bench_${TAG}_$name.log 2>&1
  local rc=$?
  echo "bench $name rc=$rc"; tail -1 $O/bench_${TAG}_$name.log
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run det python bench.py --steps 20 --warmup 3
run ens64 python bench.py --steps 5 --warmup 1 --members 64
run enkf32 python bench.py --steps 5 --warmup 1 --members 32 --enkf
run enkf256 python bench.py --steps 2 --warmup 1 --members 256 --enkf --no-cpu
run conus python bench.py --steps 3 --warmup 1 --conus
run kf python scripts/bench_kf.py
exit 0
