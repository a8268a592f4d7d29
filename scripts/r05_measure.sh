#!/bin/bash
# Round-5 measurement session: the configs[3] 8-shard emulation, the det HBM traffic of the bench
# horizons only (--no-api), det / ens64 / EnKF32 kernel stats, ens64 SQ counters.
#     bash scripts/r05_measure.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${1:-r05a}"
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u bench.py --members 256 --enkf --emulate-shards 8 --steps 2 --warmup 1 \
    --no-cpu --timing-runs 1 > $O/bench_${TAG}_enkf256_shards8.log 2>&1
rc=$?; echo "bench shards rc=$rc"; tail -c 2500 $O/bench_${TAG}_enkf256_shards8.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="" bash scripts/gpu_pmc.sh ${TAG}_det FETCH_SIZE WRITE_SIZE || exit $?
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
stats enkf32 --steps 2 --warmup 1 --members 32 --enkf
BENCH_ARGS="--members 64" bash scripts/gpu_pmc.sh ${TAG}_ens64sq \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY" || exit $?
timeout -k 10 300 python -u bench.py > $O/bench_${TAG}_det.log 2>&1
rc=$?; echo "bench det rc=$rc"; tail -c 1500 $O/bench_${TAG}_det.log; [ $rc -ne 0 ] && exit $rc
exit 0
