#!/bin/bash
# Round-5 measurement session: the N = 2 bench branch (gloo, one GPU), the configs[3] 8-shard
# emulation, the det HBM traffic of the bench horizons only (--no-api), det kernel stats.
#     bash scripts/r05_measure.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${1:-r05a}"
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 280 --timeout-method thread \
    -p no:cacheprovider tests/test_gpu_dist.py > $O/${TAG}_pytest_dist.txt 2>&1
rc=$?; echo "pytest dist rc=$rc"; tail -3 $O/${TAG}_pytest_dist.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --members 256 --enkf --emulate-shards 8 --steps 2 --warmup 1 \
    --no-cpu --timing-runs 1 > $O/bench_${TAG}_enkf256_shards8.log 2>&1
rc=$?; echo "bench shards rc=$rc"; tail -c 3000 $O/bench_${TAG}_enkf256_shards8.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="" bash scripts/gpu_pmc.sh ${TAG}_det FETCH_SIZE WRITE_SIZE || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof_${TAG}_det" \
    -o run -- python3 "$PWD/bench.py" --no-cpu --no-api --timing-runs 1 --steps 5 --warmup 1 \
    > $O/prof_${TAG}_det.log 2>&1
rc=$?; echo "stats det rc=$rc"; [ $rc -ne 0 ] && exit $rc
exit 0
