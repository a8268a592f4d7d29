# wave-uniform bound on the staging's inline gain gathers: lazy-gain / EnKF parity tests and the
# EnKF256 kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_analysis.py tests/test_gpu_configs.py tests/test_gpu_ensemble.py > gpurun_out/r05q_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05q_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_r05q_enkf256" \
    -o run -- python3 "$PWD/bench.py" --no-cpu --no-api --timing-runs 1 --steps 1 --warmup 1 --members 256 --enkf > gpurun_out/prof_r05q_enkf256.log 2>&1
rc=$?; echo "stats rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_r05q_enkf256.log)"
exit $rc
