# full GPU suite, then the det / HUC-8 / ens64 same-box A/B against round 4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_suite.sh r05l || exit $?
run() {  # tag dir args
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python -u bench.py --no-api --no-cpu "$@") > gpurun_out/r05l_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05l_$tag.log)"; [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2; do run det_cur$r . ; run det_old$r ab_r04; done
run huc8_cur . --huc8 ; run huc8_old ab_r04 --huc8
run ens64_cur . --members 64 ; run ens64_old ab_r04 --members 64
run conus_cur . --conus ; run conus_old ab_r04 --conus
exit 0
