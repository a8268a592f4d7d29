#!/bin/bash
# Round-5 closing session on the frozen build: the full GPU suite, then the profiles
# (scripts/r05m_profiles.sh: PMC traffic of det / ens64 / CONUS-16, kernel stats) under tag r05z
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_suite.sh r05z || exit $?
bash scripts/r05m_profiles.sh r05z || exit $?
exit 0
