# analysis path on the own dense kernels: parity, then EnKF bench lines and a kernel-trace profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_analysis.py tests/test_gpu_dist.py "tests/test_gpu_configs.py::test_config3_texas_enkf256_member_step_and_analysis" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03c_pytest_analysis.txt 2>&1
rc=$?; tail -15 gpurun_out/r03c_pytest_analysis.txt; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --members 256 --enkf --no-cpu > gpurun_out/r03c_bench_enkf256.json 2>&1
rc=$?; tail -c 600 gpurun_out/r03c_bench_enkf256.json; echo "bench256 rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --members 32 --enkf --no-cpu > gpurun_out/r03c_bench_enkf32.json 2>&1
rc=$?; tail -c 400 gpurun_out/r03c_bench_enkf32.json; echo "bench32 rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r03c_prof_enkf256" -o run -- python3 "$PWD/bench.py" --no-cpu --timing-runs 1 --steps 1 --warmup 1 --members 256 --enkf > gpurun_out/r03c_prof_enkf256.log 2>&1
rc=$?; echo "prof rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03c_pytest_api.txt 2>&1
rc=$?; tail -5 gpurun_out/r03c_pytest_api.txt; echo "api rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u scripts/bench_subbasins.py > gpurun_out/r03c_subbasins.json 2> gpurun_out/r03c_subbasins.err
rc=$?; cat gpurun_out/r03c_subbasins.json; tail -3 gpurun_out/r03c_subbasins.err; echo "subbasins rc=$rc"
exit $rc
