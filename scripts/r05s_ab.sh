# helper wave stores only live slot pairs: parity tests, det / HUC-8 A/B vs HEAD (ab_v1), and
# the det WRITE_SIZE pass
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_routing.py tests/test_gpu_edges.py tests/test_gpu_api.py > gpurun_out/r05s_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05s_tests.txt; [ $rc -ne 0 ] && exit $rc
run() {  # tag dir args
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python -u bench.py --no-api --no-cpu "$@") > gpurun_out/r05s_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05s_$tag.log)"; [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2; do run det_cur$r . ; run det_head$r ab_v1; done
run huc8_cur . --huc8 ; run huc8_head ab_v1 --huc8
BENCH_ARGS="" bash scripts/gpu_pmc.sh r05s_det WRITE_SIZE || exit $?
exit 0
