# multi-launch kernel in the fast form (no frozen partial sums) vs round 4: ens64, CONUS-16
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag dir args
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python -u bench.py --no-api --no-cpu "$@") > gpurun_out/r05n_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05n_$tag.log)"; [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2; do run ens64_cur$r . --members 64 ; run ens64_old$r ab_r04 --members 64; done
run conus_cur . --conus ; run conus_old ab_r04 --conus
exit 0
