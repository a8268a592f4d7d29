# same-box A/B of the det tick: current, no hi-mask (v1), act by G (v2), round 4 (ab_r04)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag dir args
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python -u bench.py --no-api --no-cpu "$@") > gpurun_out/r05k2_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05k2_$tag.log)"; [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2; do run new$r . ; run v1_$r ab_v1 ; run v2_$r ab_v2 ; run old$r ab_r04 ; done
run huc8_v1 ab_v1 --huc8 ; run huc8_new . --huc8
exit 0
