set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "det:" "ens64:--members 64" "huc8:--huc8"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python -u bench.py --no-api --cpu-seconds 2 $args > gpurun_out/r05j_bench_$name.log 2>&1
  rc=$?; echo "bench $name rc=$rc"; tail -c 300 gpurun_out/r05j_bench_$name.log | grep -o '"ms_per_step": [0-9.]*'; [ $rc -ne 0 ] && exit $rc
done
exit 0
