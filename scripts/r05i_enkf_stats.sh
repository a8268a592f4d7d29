#!/bin/bash
# EnKF256 / EnKF32 kernel stats on this build (one horizon each after one warm-up).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${1:-r05i}"
O=gpurun_out
mkdir -p $O
stats() {   # name, bench args
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof_${TAG}_$name" \
      -o run -- python3 "$PWD/bench.py" --no-cpu --no-api --timing-runs 1 "$@" > $O/prof_${TAG}_$name.log 2>&1
  local rc=$?
  echo "stats $name rc=$rc"; tail -c 400 $O/prof_${TAG}_$name.log
  [ $rc -ne 0 ] && exit $rc
  return 0
}
stats enkf256 --steps 1 --warmup 1 --members 256 --enkf
stats enkf32 --steps 1 --warmup 1 --members 32 --enkf
exit 0
