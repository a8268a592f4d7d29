# Masked output stores (only active (slot, tick) cells of a window row are written: mask) vs
# whole rows (cur): full GPU suite on mask, same-box A/B det / ens64 / CONUS-16, WRITE_SIZE of mask
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r03u_pytest_gpu.txt 2>&1
rc=$?; tail -2 $O/r03u_pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "cur mask" "--steps 20 --warmup 3" > $O/r03u_ab_det.txt 2>&1
rc=$?; cat $O/r03u_ab_det.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "cur mask" "--steps 5 --warmup 1 --members 64" > $O/r03u_ab_ens64.txt 2>&1
rc=$?; cat $O/r03u_ab_ens64.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh "cur mask" "--steps 3 --warmup 1 --conus" > $O/r03u_ab_conus.txt 2>&1
rc=$?; cat $O/r03u_ab_conus.txt; [ $rc -ne 0 ] && exit $rc
pass() {   # name, counter, bench args...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr --output-format csv \
      -d "$PWD/$O/r03u_$name" -o run -- python3 "$PWD/bench.py" --steps 1 --warmup 0 \
      --no-cpu --no-api --timing-runs 1 "$@" > $O/r03u_$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
pass det_write WRITE_SIZE
pass det_fetch FETCH_SIZE
pass ens64_write WRITE_SIZE --members 64
pass ens64_fetch FETCH_SIZE --members 64
exit 0
