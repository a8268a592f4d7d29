#!/bin/bash
# A/B of two library builds (lib/exp/lib_<name>.so) on one bench workload, same box:
#     bash scripts/ab_lib.sh "old new" "<bench args>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
E=tx-fast-hydrology_amd/tx_fast_hydrology_amd/lib/exp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in $1; do
    MCROUTE_LIB=$PWD/$E/lib_$v.so timeout -k 10 300 python bench.py --no-cpu --timing-runs 1 $2 \
        > gpurun_out/abl_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/abl_$v.log; exit 1; }
    python - gpurun_out/abl_$v.log "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "ms", round(d["ms_per_step"], 3), "kern_ms", d["roofline"]["kernel_ms_per_step"])
PY
  done
done
