#!/bin/bash
# One GPU-box profiling session for the committed profiles/ summaries:
#   kernel-trace stats of the det / ensemble / EnKF bench workloads and of the full-covariance
#   KF (scripts/bench_kf.py), HBM traffic (two PMC passes)
#   and SQ timing counters of the det workload.  Usage: bash scripts/profile_round.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${1:-r01}"
O=gpurun_out
mkdir -p $O
stats() {   # name, bench args
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof_$name" \
      -o run -- python3 "$PWD/bench.py" --no-cpu --timing-runs 1 "$@" > $O/prof_$name.log 2>&1
  local rc=$?
  echo "stats $name rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $O/prof_$name.log; exit $rc; }
  return 0
}
stats det --steps 5 --warmup 1
stats ens64 --steps 2 --warmup 1 --members 64
stats enkf32 --steps 1 --warmup 1 --members 32 --enkf
stats enkf256 --steps 1 --warmup 1 --members 256 --enkf
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof_kf" -o run \
    -- python3 "$PWD/scripts/bench_kf.py" --no-cpu --steps 1 > $O/prof_kf.log 2>&1 || exit $?
BENCH_ARGS="" bash scripts/gpu_pmc.sh ${TAG}_hbm FETCH_SIZE WRITE_SIZE || exit $?
bash scripts/gpu_pmc.sh ${TAG}_sq "SQ_WAVES SQ_WAVE_CYCLES" "SQ_BUSY_CYCLES SQ_WAIT_ANY" \
    "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
    "SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_SALU SQ_INST_CYCLES_VMEM" || exit $?
exit 0
