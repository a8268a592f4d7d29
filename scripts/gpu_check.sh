#!/bin/bash
# One GPU-box session: GPU parity tests, bench, rocprofv3 kernel-trace summary.
# Stops at the first crash / timeout (exit codes other than pytest's 0/1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${1:-r01}"
STEPS="${BENCH_STEPS:-10}"

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q --timeout=400 > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi

timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench_${TAG}.log
[ $rc -ne 0 ] && exit $rc

if [ "${SKIP_PROF:-0}" != "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_${TAG}" -o run \
      --output-format csv -- python3 "$PWD/bench.py" --steps 3 --warmup 1 --no-cpu \
      --timing-runs 1 ${BENCH_ARGS:-} > gpurun_out/prof_${TAG}.log 2>&1
  rc=$?
  echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_${TAG}.log
  find gpurun_out/prof_${TAG} -name "*stats*" | head
fi
exit $rc
