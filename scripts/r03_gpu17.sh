# member-major cells through bounds-checked buffer offsets (memb2) vs templated (memb) vs base
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_ensemble.py tests/test_gpu_analysis.py "tests/test_gpu_configs.py::test_config3_texas_enkf256_member_step_and_analysis" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03r_pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/r03r_pytest.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "base memb memb2" "--steps 5 --warmup 1 --members 32 --enkf" > gpurun_out/r03r_ab_enkf32.txt 2>&1
rc=$?; cat gpurun_out/r03r_ab_enkf32.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r03r_prof_enkf32" -o run -- python3 "$PWD/bench.py" --no-cpu --no-api --timing-runs 1 --steps 1 --warmup 1 --members 32 --enkf > gpurun_out/r03r_prof32.log 2>&1
rc=$?; echo "prof32 rc=$rc"; exit $rc
