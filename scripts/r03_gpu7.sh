# per-lane member staging runs: member parity, EnKF benches (E=32 member-major vs tick-major), profiles
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_ensemble.py tests/test_gpu_analysis.py "tests/test_gpu_configs.py::test_config3_texas_enkf256_member_step_and_analysis" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03h_pytest.txt 2>&1
rc=$?; tail -4 gpurun_out/r03h_pytest.txt; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
MCR_AB_SKEW=1 timeout -k 10 700 python -u -m pytest tests/test_gpu_ensemble.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03h_pytest_skew.txt 2>&1
rc=$?; tail -2 gpurun_out/r03h_pytest_skew.txt; echo "pytest skew rc=$rc"
[ $rc -ne 0 ] && exit $rc
for v in 128 1 128 1; do
  MCR_AB_SKEW=$v timeout -k 10 300 python bench.py --steps 5 --warmup 1 --members 32 --enkf --no-cpu > gpurun_out/r03h_enkf32_s$v.json 2>&1
  rc=$?; echo "E=32 skew>=$v rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/r03h_enkf32_s$v.json').read().strip().splitlines()[-1]);print(round(d['ms_per_horizon'],2))")"
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --members 256 --enkf --no-cpu > gpurun_out/r03h_enkf256.json 2>&1
rc=$?; echo "E=256 rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/r03h_enkf256.json').read().strip().splitlines()[-1]);print(round(d['ms_per_horizon'],2))")"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r03h_prof_enkf256" -o run -- python3 "$PWD/bench.py" --no-cpu --timing-runs 1 --steps 1 --warmup 1 --members 256 --enkf > gpurun_out/r03h_prof.log 2>&1
rc=$?; echo "prof256 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r03h_prof_enkf32" -o run -- python3 "$PWD/bench.py" --no-cpu --timing-runs 1 --steps 2 --warmup 1 --members 32 --enkf > gpurun_out/r03h_prof32.log 2>&1
rc=$?; echo "prof32 rc=$rc"
exit $rc
