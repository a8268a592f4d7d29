# Forcing prefetch only for slots that run in the next chunk (fl) vs live: ensemble / config
# parity on fl, same-box A/B ens64 / CONUS-16
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ensemble.py tests/test_gpu_configs.py tests/test_gpu_routing.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r03x_pytest.txt 2>&1
rc=$?; tail -2 $O/r03x_pytest.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "live fl" "--steps 5 --warmup 1 --members 64" > $O/r03x_ab_ens64.txt 2>&1
rc=$?; cat $O/r03x_ab_ens64.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "live fl" "--steps 3 --warmup 1 --conus" > $O/r03x_ab_conus.txt 2>&1
rc=$?; cat $O/r03x_ab_conus.txt; [ $rc -ne 0 ] && exit $rc
exit 0
