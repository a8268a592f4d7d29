set -u
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_ensemble.py -k "single_steps or matches_launches or copy_state" > gpurun_out/r05g_pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r05g_pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --members 32 --enkf --steps 3 --warmup 1 --no-cpu --timing-runs 1 > gpurun_out/r05g_enkf32_paths.log 2>&1
rc=$?; echo "bench paths rc=$rc"; tail -c 600 gpurun_out/r05g_enkf32_paths.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --members 32 --enkf --steps 3 --warmup 1 --no-cpu --timing-runs 1 --mode dataflow > gpurun_out/r05g_enkf32_dataflow.log 2>&1
rc=$?; echo "bench dataflow rc=$rc"; tail -c 300 gpurun_out/r05g_enkf32_dataflow.log
exit $rc
