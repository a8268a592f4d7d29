# first-chunk forcing loads issued with the slot registers (this tree) vs HEAD (ab_v1): the
# multi-launch parity tests, then ens64 / CONUS-16 on the same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_routing.py tests/test_gpu_configs.py tests/test_gpu_edges.py -k "launches or config or ens or member" > gpurun_out/r05r_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05r_tests.txt; [ $rc -ne 0 ] && exit $rc
run() {  # tag dir args
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python -u bench.py --no-api --no-cpu "$@") > gpurun_out/r05r_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05r_$tag.log)"; [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2; do run ens64_cur$r . --members 64 ; run ens64_head$r ab_v1 --members 64; done
run conus_cur . --conus ; run conus_head ab_v1 --conus
exit 0
