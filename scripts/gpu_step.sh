# round results on the GPU box: PART=1 tests + smoke + bench lines, PART=2 rocprof profiles
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r06b}
if [ "${PART:-1}" = 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${T}.txt 2>&1 || { tail -20 gpurun_out/pytest_${T}.txt; exit 1; }
tail -2 gpurun_out/pytest_${T}.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${T}.log 2>&1 || exit 1
bash scripts/bench_round.sh $T || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --huc8 > gpurun_out/bench_${T}_huc8.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --members 256 --enkf --no-cpu --emulate-shards 8 > gpurun_out/bench_${T}_enkf256_shards.log 2>&1 || exit 1
else
bash scripts/round_profiles.sh $T || exit 1
fi
