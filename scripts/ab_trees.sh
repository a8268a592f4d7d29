#!/bin/bash
# A/B of the current tree against ab_old/ (an older tree with its own library) on one box:
#     bash scripts/ab_trees.sh "<bench args>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for t in old new; do
    d=.; [ $t = old ] && d=${AB_OLD:-ab_old}
    (cd $d && timeout -k 10 300 python bench.py --no-cpu --timing-runs 1 $1) > gpurun_out/abt_$t.log 2>&1 \
        || { echo "$t failed"; tail -3 gpurun_out/abt_$t.log; exit 1; }
    python - gpurun_out/abt_$t.log $t <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "ms", round(d["ms_per_step"], 3), "kern_ms", d["roofline"]["kernel_ms_per_step"],
      "launches", d["roofline"]["launches_per_step"], "ticks", d["config"]["schedule_ticks"], "nwg", d["config"]["nwg"])
PY
  done
done
