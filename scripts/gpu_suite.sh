#!/bin/bash
# The full GPU test suite on one box (own time limit), output under gpurun_out/<tag>_pytest_gpu.txt
#     bash scripts/gpu_suite.sh <tag> [pytest args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="${1:-r05}"
shift || true
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu ${PYTEST_X:--x} -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider "${@:-tests}" > gpurun_out/${TAG}_pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/${TAG}_pytest_gpu.txt
exit $rc
