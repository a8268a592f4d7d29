# EnKF256 member steps: member-major cells with the buffer-addressed member kernel (noskew) vs
# tick-major windows (cur)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/ab_lib.sh "cur noskew" "--steps 3 --warmup 1 --members 256 --enkf" > gpurun_out/r03s_ab_enkf256.txt 2>&1
rc=$?; cat gpurun_out/r03s_ab_enkf256.txt; [ $rc -ne 0 ] && exit $rc
MCROUTE_LIB=$PWD/tx-fast-hydrology_amd/tx_fast_hydrology_amd/lib/exp/lib_noskew.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r03s_prof_noskew" -o run -- python3 "$PWD/bench.py" --no-cpu --no-api --timing-runs 1 --steps 1 --warmup 1 --members 256 --enkf > gpurun_out/r03s_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
