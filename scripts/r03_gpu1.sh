set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_gpu.txt 2>&1
rc=$?; tail -5 gpurun_out/r03_pytest_gpu.txt; echo "pytest rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/r03_bench_det.json 2> gpurun_out/r03_bench_det.err
rc2=$?; tail -c 3000 gpurun_out/r03_bench_det.json; echo "bench rc=$rc2"
exit $rc
