# is the fast form taken?  this tree vs exact forced off (ab_v1) vs partial-sum form removed (ab_v2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag dir args
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python -u bench.py --no-api --no-cpu "$@") > gpurun_out/r05k10_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05k10_$tag.log)"; [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2; do run det_cur$r . ; run det_fast$r ab_v1 ; run det_old$r ab_r04; done
exit 0
