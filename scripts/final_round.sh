#!/bin/bash
# The round's closing GPU session on the frozen build, most important first: the full GPU test
# suite, HBM traffic (det / ens64 / CONUS-16), kernel stats (EnKF256, EnKF32, det, ens64), bench
# lines (EnKF256 with the 8-shard emulation, det, EnKF32, ens64, CONUS-16, HUC-8), smoke.
# Every step has its own time limit; the session stops at the first failure.
#     bash scripts/final_round.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${1:-r04}"
O=gpurun_out
mkdir -p $O
timeout -k 10 420 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider tests > $O/${TAG}_pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/${TAG}_pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
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
stats enkf256 --steps 1 --warmup 1 --members 256 --enkf
stats enkf32 --steps 1 --warmup 1 --members 32 --enkf
stats det --steps 5 --warmup 1
stats ens64 --steps 2 --warmup 1 --members 64
run() {   # name, command...
  local name=$1; shift
  timeout -k 10 300 "$@" > $O/bench_${TAG}_$name.log 2>&1
  local rc=$?
  echo "bench $name rc=$rc"; tail -1 $O/bench_${TAG}_$name.log
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run enkf256 python bench.py --steps 2 --warmup 1 --members 256 --enkf --emulate-shards 8 --cpu-seconds 10
run det python bench.py --steps 20 --warmup 3
run enkf32 python bench.py --steps 5 --warmup 1 --members 32 --enkf
run ens64 python bench.py --steps 5 --warmup 1 --members 64
run conus python bench.py --steps 3 --warmup 1 --conus
run huc8 python bench.py --huc8
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"
exit $rc
