# tick-major member staging: member parity, EnKF benches, profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_ensemble.py tests/test_gpu_analysis.py tests/test_gpu_dist.py "tests/test_gpu_configs.py::test_config3_texas_enkf256_member_step_and_analysis" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03g_pytest.txt 2>&1
rc=$?; tail -4 gpurun_out/r03g_pytest.txt; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for E in 32 256; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --members $E --enkf --no-cpu > gpurun_out/r03g_enkf$E.json 2>&1
  rc=$?; echo "E=$E rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/r03g_enkf$E.json').read().strip().splitlines()[-1]);print(round(d['ms_per_horizon'],2))")"
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r03g_prof_enkf256" -o run -- python3 "$PWD/bench.py" --no-cpu --timing-runs 1 --steps 1 --warmup 1 --members 256 --enkf > gpurun_out/r03g_prof.log 2>&1
rc=$?; echo "prof rc=$rc"
exit $rc
