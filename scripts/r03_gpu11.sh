# output rows by path (hC: segment rows for the det dataflow horizon, workgroup rows with the
# round-2 store code for the multi-launch kernel) vs the round-start build (old); layout parity
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/ab_lib.sh "old hC" "--steps 5 --warmup 1 --members 64" > gpurun_out/r03l_ab_ens64.txt 2>&1
rc=$?; cat gpurun_out/r03l_ab_ens64.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "old hC" "--steps 20 --warmup 3 --no-api" > gpurun_out/r03l_ab_det.txt 2>&1
rc=$?; cat gpurun_out/r03l_ab_det.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_routing.py tests/test_gpu_ensemble.py tests/test_gpu_api.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03l_pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/r03l_pytest.txt; exit $rc
