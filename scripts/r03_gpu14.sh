# final build check: GPU suite + smoke, HUC-8 lane shapes, then the part-B evidence again
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r03z_pytest_gpu.txt 2>&1
rc=$?; tail -2 $O/r03z_pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r03z_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
for sc in "192 2" "384 2" "448 2" "192 3" "256 3" "192 4" "128 4"; do
  set -- $sc
  timeout -k 10 120 python bench.py --huc8 --steps 50 --warmup 5 --no-cpu --no-api --slots $1 --chain $2 > $O/r03o_huc8_$1_$2.json 2>&1
  rc=$?; echo "huc8 slots=$1 chain=$2 rc=$rc $(python -c "import json;d=json.loads(open('$O/r03o_huc8_$1_$2.json').read().strip().splitlines()[-1]);print(round(d['ms_per_horizon'],4), d['config']['nwg'], d['config']['schedule_ticks'], d['roofline']['avg_launch_us'])" 2>&1 | tail -1)"
done
bash scripts/r03_final_b.sh
exit $?
