# lane shapes for small single-member networks: 1 compute wave x 1 slot vs the 192 x 2 default
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag args
  local tag=$1; shift
  timeout -k 10 200 python -u bench.py --no-api --no-cpu --steps 10 --warmup 2 "$@" > gpurun_out/r05v_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05v_$tag.log) $(grep -o '"launches_per_step": [0-9.]*' gpurun_out/r05v_$tag.log) $(grep -o '"schedule_ticks": [0-9]*' gpurun_out/r05v_$tag.log | head -1) $(grep -o '"nwg": [0-9]*' gpurun_out/r05v_$tag.log | head -1)"
  return 0
}
for n in 4000 12000 30000; do
  d=$((n / 20)); b=$((n / 2000 + 1))
  run n${n}_64x1 --n $n --basins $b --depth $d --slots 64 --chain 1
  run n${n}_64x2 --n $n --basins $b --depth $d --slots 64 --chain 2
  run n${n}_192x2 --n $n --basins $b --depth $d --slots 192 --chain 2
done
exit 0
