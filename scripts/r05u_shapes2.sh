# one-compute-wave workgroups (64 lanes) for Texas det, and HUC-8 at 64 lanes with longer tiles
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag args
  local tag=$1; shift
  timeout -k 10 200 python -u bench.py --no-api --no-cpu --steps 10 --warmup 2 "$@" > gpurun_out/r05u2_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05u2_$tag.log) $(grep -o '"launches_per_step": [0-9.]*' gpurun_out/r05u2_$tag.log) $(grep -o '"schedule_ticks": [0-9]*' gpurun_out/r05u2_$tag.log | head -1) $(grep -o '"nwg": [0-9]*' gpurun_out/r05u2_$tag.log | head -1)"
  return 0
}
run det_64x2 --slots 64 ; run det_64x3 --slots 64 --chain 3 ; run det_64x4 --slots 64 --chain 4
run huc8_64x2_t24 --huc8 --slots 64 --tile 24 ; run huc8_64x2_r --huc8 --slots 64 ; run huc8_64x1 --huc8 --slots 64 --chain 1 ; run huc8_192x2_r --huc8
exit 0
