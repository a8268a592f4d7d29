#!/bin/bash
# Bench lines of the round-5 build (each its own time limit) and the smoke
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="${1:-r05m}"
O=gpurun_out
mkdir -p $O
run() {   # name, command...
  local name=$1; shift
  timeout -k 10 300 "$@" > $O/bench_${TAG}_$name.log 2>&1
  local rc=$?
  echo "bench $name rc=$rc"; grep -o '"ms_per_step": [0-9.]*' $O/bench_${TAG}_$name.log | head -1
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run det python bench.py --steps 20 --warmup 3
run huc8 python bench.py --huc8
run ens64 python bench.py --steps 5 --warmup 1 --members 64
run enkf32 python bench.py --steps 5 --warmup 1 --members 32 --enkf
run enkf256 python bench.py --steps 2 --warmup 1 --members 256 --enkf --emulate-shards 8 --cpu-seconds 10
run conus python bench.py --steps 3 --warmup 1 --conus
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"
exit $rc
