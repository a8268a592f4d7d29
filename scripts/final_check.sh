# final build on the GPU box: the GPU suite, smoke, the det bench line, and the profiles whose
# source hash the bench lines check (PMC traffic det / ens64 / CONUS-16, kernel stats)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r06d}
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${T}.txt 2>&1 || { tail -20 gpurun_out/pytest_${T}.txt; exit 1; }
tail -1 gpurun_out/pytest_${T}.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${T}.log 2>&1 || exit 1
BENCH_ARGS="" bash scripts/gpu_pmc.sh ${T}_det FETCH_SIZE WRITE_SIZE || exit $?
BENCH_ARGS="--members 64" bash scripts/gpu_pmc.sh ${T}_ens64 FETCH_SIZE WRITE_SIZE || exit $?
BENCH_ARGS="--conus" bash scripts/gpu_pmc.sh ${T}_conus FETCH_SIZE WRITE_SIZE || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_${T}_det" \
    -o run -- python3 "$PWD/bench.py" --no-cpu --no-api --timing-runs 1 --steps 5 --warmup 1 > gpurun_out/prof_${T}_det.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_${T}_det.log 2>&1 || exit 1
tail -1 gpurun_out/bench_${T}_det.log | cut -c1-300
