# the fast / exact partial-sum forms: parity tests, then det / HUC-8 / ens64 against round 4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag dir args
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python -u bench.py --no-api --no-cpu "$@") > gpurun_out/r05k9_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05k9_$tag.log)"; [ $rc -ne 0 ] && exit $rc
  return 0
}
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_edges.py tests/test_gpu_routing.py tests/test_gpu_api.py > gpurun_out/r05k9_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05k9_tests.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do run det_cur$r . ; run det_old$r ab_r04; done
run huc8_cur . --huc8 ; run huc8_old ab_r04 --huc8
run ens64_cur . --members 64 ; run ens64_old ab_r04 --members 64
exit 0
