# member kernel templated on the staging layout (memb) vs base: member parity, EnKF A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_ensemble.py "tests/test_gpu_configs.py::test_config3_texas_enkf256_member_step_and_analysis" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03q_pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/r03q_pytest.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "base memb" "--steps 5 --warmup 1 --members 32 --enkf" > gpurun_out/r03q_ab_enkf32.txt 2>&1
rc=$?; cat gpurun_out/r03q_ab_enkf32.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "base memb" "--steps 3 --warmup 1 --members 256 --enkf" > gpurun_out/r03q_ab_enkf256.txt 2>&1
rc=$?; cat gpurun_out/r03q_ab_enkf256.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r03q_prof_enkf32" -o run -- python3 "$PWD/bench.py" --no-cpu --no-api --timing-runs 1 --steps 1 --warmup 1 --members 32 --enkf > gpurun_out/r03q_prof32.log 2>&1
rc=$?; echo "prof32 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r03q_prof_enkf256" -o run -- python3 "$PWD/bench.py" --no-cpu --no-api --timing-runs 1 --steps 1 --warmup 1 --members 256 --enkf > gpurun_out/r03q_prof256.log 2>&1
rc=$?; echo "prof256 rc=$rc"; exit $rc
