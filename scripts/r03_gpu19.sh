# fused gauge prep + single-block SPD solve (fuse) vs cur: analysis parity, EnKF32 A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MCROUTE_LIB=$PWD/tx-fast-hydrology_amd/tx_fast_hydrology_amd/lib/exp/lib_fuse.so timeout -k 10 700 python -u -m pytest tests/test_gpu_analysis.py tests/test_gpu_dist.py tests/test_gpu_kalman.py "tests/test_gpu_configs.py::test_config3_texas_enkf256_member_step_and_analysis" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03t_pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/r03t_pytest.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "cur fuse" "--steps 5 --warmup 1 --members 32 --enkf" > gpurun_out/r03t_ab_enkf32.txt 2>&1
rc=$?; cat gpurun_out/r03t_ab_enkf32.txt; [ $rc -ne 0 ] && exit $rc
for sc in "256 64" "256 32" "192 64" "128 64" "256 64"; do
  set -- $sc
  timeout -k 10 200 python bench.py --members 32 --enkf --steps 5 --warmup 1 --no-cpu --fslots $1 --ftile $2 > gpurun_out/r03t_enkf32_f$1_$2.json 2>&1
  rc=$?; echo "enkf32 forecast slots=$1 tile=$2 rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/r03t_enkf32_f$1_$2.json').read().strip().splitlines()[-1]);print(round(d['ms_per_horizon'],3))" 2>&1 | tail -1)"
done
exit 0
