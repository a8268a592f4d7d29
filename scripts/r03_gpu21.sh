# Live-slot state stores in the multi-launch kernel (live = mask + state written only for slots
# that ran in the launch) vs mask vs cur: full GPU suite on live, same-box A/B ens64 / CONUS-16 /
# EnKF32
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r03v_pytest_gpu.txt 2>&1
rc=$?; tail -2 $O/r03v_pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "cur mask live" "--steps 5 --warmup 1 --members 64" > $O/r03v_ab_ens64.txt 2>&1
rc=$?; cat $O/r03v_ab_ens64.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "cur live" "--steps 3 --warmup 1 --conus" > $O/r03v_ab_conus.txt 2>&1
rc=$?; cat $O/r03v_ab_conus.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "cur live" "--steps 5 --warmup 1 --members 32 --enkf" > $O/r03v_ab_enkf32.txt 2>&1
rc=$?; cat $O/r03v_ab_enkf32.txt; [ $rc -ne 0 ] && exit $rc
exit 0
