# members per multi-launch instance (MCR_MPI): ensemble parity tests at 1 and 3 members per
# instance, then ens64 / CONUS-16 at 1, 2, 4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in 1 3; do
  MCR_MPI=$m timeout -k 10 500 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_ensemble.py tests/test_gpu_configs.py tests/test_gpu_edges.py -k "not paths" > gpurun_out/r05t_tests_$m.txt 2>&1
  rc=$?; echo "tests mpi=$m rc=$rc"; tail -1 gpurun_out/r05t_tests_$m.txt; [ $rc -ne 0 ] && exit $rc
done
run() {  # tag mpi args
  local tag=$1 m=$2; shift 2
  MCR_MPI=$m timeout -k 10 300 python -u bench.py --no-api --no-cpu "$@" > gpurun_out/r05t_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05t_$tag.log)"; [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2; do run ens64_m1_$r 1 --members 64 ; run ens64_m2_$r 2 --members 64 ; run ens64_m4_$r 4 --members 64; done
run conus_m1 1 --conus ; run conus_m2 2 --conus ; run conus_m4 4 --conus
exit 0
