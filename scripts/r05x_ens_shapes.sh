# lane / tile shapes of the ensemble forecast (ens64) and the EnKF32 cycle on the final build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag args
  local tag=$1; shift
  timeout -k 10 200 python -u bench.py --no-api --no-cpu --timing-runs 1 "$@" > gpurun_out/r05x_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05x_$tag.log)"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run ens64_256x64 --members 64 --steps 3 --warmup 1
run ens64_192x64 --members 64 --steps 3 --warmup 1 --slots 192
run ens64_384x64 --members 64 --steps 3 --warmup 1 --slots 384
run ens64_256x128 --members 64 --steps 3 --warmup 1 --tile 128
run ens64_256x32 --members 64 --steps 3 --warmup 1 --tile 32
run enkf32_base --members 32 --enkf --steps 3 --warmup 1
run enkf32_s128 --members 32 --enkf --steps 3 --warmup 1 --slots 128
run enkf32_s256 --members 32 --enkf --steps 3 --warmup 1 --slots 256
run enkf32_f384 --members 32 --enkf --steps 3 --warmup 1 --fslots 384
run enkf32_ft128 --members 32 --enkf --steps 3 --warmup 1 --ftile 128
exit 0
