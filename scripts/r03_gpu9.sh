# A/B segment windows (new) vs workgroup windows (old) on det and ens64; slice prefetch (pf) vs
# new on EnKF256; analysis parity with the prefetch build; API path breakdown
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_analysis.py tests/test_gpu_dist.py "tests/test_gpu_configs.py::test_config3_texas_enkf256_member_step_and_analysis" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03j_pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/r03j_pytest.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "new pf" "--steps 3 --warmup 1 --members 256 --enkf" > gpurun_out/r03j_ab_enkf256.txt 2>&1
rc=$?; cat gpurun_out/r03j_ab_enkf256.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r03j_prof_enkf256" -o run -- python3 "$PWD/bench.py" --no-cpu --timing-runs 1 --steps 1 --warmup 1 --members 256 --enkf > gpurun_out/r03j_prof.log 2>&1
rc=$?; echo "prof256 rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "old new" "--steps 20 --warmup 3 --no-api" > gpurun_out/r03j_ab_det.txt 2>&1
rc=$?; cat gpurun_out/r03j_ab_det.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "old new" "--steps 5 --warmup 1 --members 64" > gpurun_out/r03j_ab_ens64.txt 2>&1
rc=$?; cat gpurun_out/r03j_ab_ens64.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/api_breakdown.py > gpurun_out/r03j_api.json 2>&1
rc=$?; tail -2 gpurun_out/r03j_api.json; exit $rc
