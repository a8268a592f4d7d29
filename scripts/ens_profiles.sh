#!/bin/bash
# Ensemble roofline evidence: HBM traffic (two PMC passes each) and kernel-trace stats for the
# ens64 (configs[2]) and CONUS 16-member (configs[4]) bench workloads.
#   bash scripts/ens_profiles.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${1:-r01d}"
pass() {   # name, counter, bench args...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr --output-format csv \
      -d "$PWD/gpurun_out/${TAG}_$name" -o run -- python3 "$PWD/bench.py" --steps 1 --warmup 0 \
      --no-cpu --timing-runs 1 "$@" > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
pass ens64_fetch FETCH_SIZE --members 64
pass ens64_write WRITE_SIZE --members 64
pass conus_fetch FETCH_SIZE --conus
pass conus_write WRITE_SIZE --conus
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}_conus" -o run \
    --output-format csv -- python3 "$PWD/bench.py" --steps 2 --warmup 1 --no-cpu \
    --timing-runs 1 --conus > gpurun_out/prof_${TAG}_conus.log 2>&1
rc=$?
echo "rocprof conus rc=$rc"; tail -1 gpurun_out/prof_${TAG}_conus.log
exit $rc
