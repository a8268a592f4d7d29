# same-box A/B of the lateral-inflow placement: batched per chunk with a clamp branch (this
# tree), per tick with an unconditional mask (ab_v1), per tick with the clamp branch (ab_v2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag dir args
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python -u bench.py --no-api --no-cpu "$@") > gpurun_out/r05k4_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05k4_$tag.log)"; [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2; do run det_cur$r . ; run det_v1_$r ab_v1 ; run det_v2_$r ab_v2 ; run det_v3_$r ab_v3 ; run det_old$r ab_r04; done
run ens64_cur . --members 64 ; run ens64_v1 ab_v1 --members 64 ; run ens64_v2 ab_v2 --members 64 ; run ens64_v3 ab_v3 --members 64 ; run ens64_old ab_r04 --members 64
exit 0
