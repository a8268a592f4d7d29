# same-box A/B: this build vs the round-4 tree (ab_r04, a git worktree of d0f8a10)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag dir args
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python -u bench.py --no-api --no-cpu "$@") > gpurun_out/r05k_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05k_$tag.log)"; [ $rc -ne 0 ] && exit $rc
  return 0
}
run det_new . ; run det_old ab_r04 ; run det_new2 . ; run det_old2 ab_r04
run huc8_new . --huc8 ; run huc8_old ab_r04 --huc8
run ens64_new . --members 64 ; run ens64_old ab_r04 --members 64
exit 0
