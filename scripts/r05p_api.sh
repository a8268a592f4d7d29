# the fetch ring on its own copy stream: async-fetch / API parity tests, the API breakdown, the
# det bench line's api_ms_per_horizon
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_api.py tests/test_gpu_routing.py -k "async or api or simulate or fetch or golden" > gpurun_out/r05p_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05p_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/api_breakdown.py > gpurun_out/r05p_api_breakdown.txt 2>&1
rc=$?; echo "breakdown rc=$rc"; tail -1 gpurun_out/r05p_api_breakdown.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r05p_bench_det.log 2>&1
rc=$?; echo "bench rc=$rc $(grep -o '"api_ms_per_horizon": [0-9.]*' gpurun_out/r05p_bench_det.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05p_bench_det.log)"
exit $rc
