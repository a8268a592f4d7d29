# segment output windows: full GPU suite, det + ens64 benches, WRITE/FETCH PMC passes for both;
# 256-member slice tiles vs 128 (EnKF256 A/B)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03i_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r03i_pytest.txt; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-api > gpurun_out/r03i_det.json 2>&1
rc=$?; echo "det rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/r03i_det.json').read().strip().splitlines()[-1]);print(round(d['ms_per_horizon'],4))")"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --members 64 --no-cpu > gpurun_out/r03i_ens64.json 2>&1
rc=$?; echo "ens64 rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/r03i_ens64.json').read().strip().splitlines()[-1]);print(round(d['ms_per_horizon'],3))")"
[ $rc -ne 0 ] && exit $rc
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export MCR_AB_SLICE2=1; else unset MCR_AB_SLICE2; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --members 256 --enkf --no-cpu > gpurun_out/r03i_enkf256_s$v.json 2>&1
  rc=$?; echo "E=256 slice128=$v rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/r03i_enkf256_s$v.json').read().strip().splitlines()[-1]);print(round(d['ms_per_horizon'],2))")"
  [ $rc -ne 0 ] && exit $rc
done
unset MCR_AB_SLICE2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r03i_prof_enkf256" -o run -- python3 "$PWD/bench.py" --no-cpu --timing-runs 1 --steps 1 --warmup 1 --members 256 --enkf > gpurun_out/r03i_prof.log 2>&1
rc=$?; echo "prof256 rc=$rc"; [ $rc -ne 0 ] && exit $rc
for W in det ens64; do
  A="--no-api"; [ $W = ens64 ] && A="--members 64"
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$PWD/gpurun_out/r03i_pmc_${W}_$C" -o run -- python3 "$PWD/bench.py" --steps 1 --warmup 0 --no-cpu --timing-runs 1 $A > gpurun_out/r03i_pmc_${W}_$C.log 2>&1
    rc=$?; echo "pmc $W $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
python scripts/hbm_traffic.py gpurun_out/r03i_pmc_det_FETCH_SIZE gpurun_out/r03i_pmc_det_WRITE_SIZE r03i 192 16 190000 288 && \
python scripts/hbm_traffic.py gpurun_out/r03i_pmc_ens64_FETCH_SIZE gpurun_out/r03i_pmc_ens64_WRITE_SIZE r03i 256 64 190000 288 64 && \
mkdir -p gpurun_out/prof_copy && cp profiles/r03i_hbm_traffic*.json gpurun_out/prof_copy/
exit $?
