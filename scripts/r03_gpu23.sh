# Dataflow helper row copies skipped per 128-column group when no slot of the group runs at the
# tick (grp: scalar test, wave-uniform) vs whole rows (cur): det parity on grp, same-box det A/B,
# WRITE_SIZE of grp
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_routing.py tests/test_gpu_api.py tests/test_gpu_edges.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r03y_pytest.txt 2>&1
rc=$?; tail -2 $O/r03y_pytest.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "cur grp" "--steps 20 --warmup 3" > $O/r03y_ab_det.txt 2>&1
rc=$?; cat $O/r03y_ab_det.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "cur grp" "--steps 20 --warmup 3" >> $O/r03y_ab_det.txt 2>&1
rc=$?; cat $O/r03y_ab_det.txt; [ $rc -ne 0 ] && exit $rc
MCROUTE_LIB=$PWD/tx-fast-hydrology_amd/tx_fast_hydrology_amd/lib/exp/lib_grp.so timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv \
    -d "$PWD/$O/r03y_det_write" -o run -- python3 "$PWD/bench.py" --steps 1 --warmup 0 \
    --no-cpu --no-api --timing-runs 1 > $O/r03y_det_write.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
