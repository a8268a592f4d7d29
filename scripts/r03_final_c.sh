# Round-3 evidence on the masked-store build, part A (as r03_final_a.sh): GPU suite, smoke,
# every bench line of the round (CPU baselines included), the sub-basin / KF timings.  Outputs gpurun_out/r03w_*.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r03w_pytest_gpu.txt 2>&1
rc=$?; tail -2 $O/r03w_pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r03w_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/r03w_smoke.log; [ $rc -ne 0 ] && exit $rc
run() {   # name, bench args
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > $O/r03w_bench_$name.json 2>&1
  local rc=$?
  echo "bench $name rc=$rc $(python -c "import json,sys;d=json.loads(open('$O/r03w_bench_$name.json').read().strip().splitlines()[-1]);print(round(d['ms_per_horizon'],4), '%.3g'%d['value'], (d.get('cpu_baseline') or {}).get('value'))" 2>&1 | tail -1)"
  [ $rc -ne 0 ] && { tail -5 $O/r03w_bench_$name.json; exit $rc; }
  return 0
}
run det --steps 20 --warmup 3
run huc8 --huc8 --steps 50 --warmup 5
run ens64 --steps 5 --warmup 1 --members 64
run enkf32 --steps 5 --warmup 1 --members 32 --enkf
run enkf256 --steps 3 --warmup 1 --members 256 --enkf
run conus --steps 3 --warmup 1 --conus
timeout -k 10 300 python scripts/bench_subbasins.py > $O/r03w_subbasins.json 2>&1
rc=$?; echo "subbasins rc=$rc"; tail -1 $O/r03w_subbasins.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/bench_kf.py > $O/r03w_bench_kf.json 2>&1
rc=$?; echo "kf rc=$rc"; tail -1 $O/r03w_bench_kf.json
exit $rc
