# ensemble forecast plan shapes (ens64 and CONUS-16): launch length (tile) and lanes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for sc in "256 64" "256 128" "256 96" "192 64" "384 64" "256 64"; do
  set -- $sc
  timeout -k 10 200 python bench.py --members 64 --steps 5 --warmup 1 --no-cpu --slots $1 --tile $2 > $O/r03p_ens64_$1_$2.json 2>&1
  rc=$?; echo "ens64 slots=$1 tile=$2 rc=$rc $(python -c "import json;d=json.loads(open('$O/r03p_ens64_$1_$2.json').read().strip().splitlines()[-1]);print(round(d['ms_per_horizon'],3), d['config']['nwg'], d['config']['schedule_ticks'], d['roofline']['launches_per_step'])" 2>&1 | tail -1)"
done
for sc in "256 64" "256 128"; do
  set -- $sc
  timeout -k 10 300 python bench.py --conus --steps 3 --warmup 1 --no-cpu --slots $1 --tile $2 > $O/r03p_conus_$1_$2.json 2>&1
  rc=$?; echo "conus slots=$1 tile=$2 rc=$rc $(python -c "import json;d=json.loads(open('$O/r03p_conus_$1_$2.json').read().strip().splitlines()[-1]);print(round(d['ms_per_horizon'],3), d['config']['schedule_ticks'], d['roofline']['launches_per_step'])" 2>&1 | tail -1)"
done
exit 0
