#!/bin/bash
# PMC counter passes for the wavefront kernel (counters only with --kernel-trace, one group per pass).
# --no-api: the pass must record the bench horizons only (scripts/hbm_traffic.py refuses a mixed set)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${1:-pmc}"
shift || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv \
      -d "$PWD/gpurun_out/${TAG}_p$i" -o run -- python3 "$PWD/bench.py" --steps 1 --warmup 0 \
      --no-cpu --no-api --timing-runs 1 ${BENCH_ARGS:-} > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "pmc pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
