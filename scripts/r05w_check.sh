# size-aware default shape of single-member sessions: full GPU suite, HUC-8 bench line, the
# sub-basin DAG timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_suite.sh r05w || exit $?
timeout -k 10 300 python -u bench.py --huc8 --cpu-seconds 3 > gpurun_out/r05w_bench_huc8.log 2>&1
rc=$?; echo "huc8 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05w_bench_huc8.log) $(grep -o '"frac": [0-9.]*' gpurun_out/r05w_bench_huc8.log | head -3 | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/bench_subbasins.py --runs 2 > gpurun_out/r05w_subbasins.txt 2>&1
rc=$?; echo "subbasins rc=$rc"; tail -c 600 gpurun_out/r05w_subbasins.txt
exit $rc
