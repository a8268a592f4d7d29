# Round-end check of the tree as left (in-tree library rebuilt from the r03w sources): GPU suite,
# smoke, default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r03_end_pytest_gpu.txt 2>&1
rc=$?; tail -2 $O/r03_end_pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r03_end_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/r03_end_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $O/r03_end_bench.json 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 $O/r03_end_bench.json; exit $rc
