set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_ensemble.py tests/test_gpu_analysis.py -k "single_steps or matches_launches or lazy_gain" > gpurun_out/r05h_pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r05h_pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/diag_paths.py > gpurun_out/r05h_diag.txt 2>&1
rc=$?; echo "diag rc=$rc"; grep -v amdgpu.ids gpurun_out/r05h_diag.txt | tail -20
exit $rc
