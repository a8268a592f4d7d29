# lane shapes of the det and HUC-8 dataflow launches on this build (168 VGPRs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag args
  local tag=$1; shift
  timeout -k 10 200 python -u bench.py --no-api --no-cpu --steps 10 --warmup 2 "$@" > gpurun_out/r05u_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05u_$tag.log) $(grep -o '"launches_per_step": [0-9.]*' gpurun_out/r05u_$tag.log) $(grep -o '"schedule_ticks": [0-9]*' gpurun_out/r05u_$tag.log | head -1) $(grep -o '"nwg": [0-9]*' gpurun_out/r05u_$tag.log | head -1)"
  return 0
}
run det_192x2 ; run det_128x2 --slots 128 ; run det_128x3 --slots 128 --chain 3 ; run det_192x3 --slots 192 --chain 3 ; run det_256x2 --slots 256
run huc8_192x2 --huc8 ; run huc8_64x2 --huc8 --slots 64 ; run huc8_128x2 --huc8 --slots 128 ; run huc8_64x3 --huc8 --slots 64 --chain 3
exit 0
