# output rows per session: segment rows for det, workgroup rows for ensembles (hA: generic
# per-position cells, hB: + one workgroup row test); A/B vs old (workgroup windows) / new
# (segments everywhere); then routing/ensemble/API parity on hB
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/ab_lib.sh "old new hA hB" "--steps 5 --warmup 1 --members 64" > gpurun_out/r03k_ab_ens64.txt 2>&1
rc=$?; cat gpurun_out/r03k_ab_ens64.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "old hB" "--steps 20 --warmup 3 --no-api" > gpurun_out/r03k_ab_det.txt 2>&1
rc=$?; cat gpurun_out/r03k_ab_det.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_routing.py tests/test_gpu_ensemble.py tests/test_gpu_api.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03k_pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/r03k_pytest.txt; exit $rc
