#!/bin/bash
# Texas det horizon at several (chain, slots) plan shapes on one GPU box:
#     bash scripts/chain_bench.sh "2:192 3:192 4:192 4:256"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cs in ${1:-2:192 4:192}; do
  c=${cs%%:*}; sl=${cs#*:}
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --timing-runs 3 --chain $c \
      --slots $sl ${BENCH_ARGS:-} > gpurun_out/cb_${c}_${sl}.log 2>&1 \
      || { echo "chain $c slots $sl failed"; tail -3 gpurun_out/cb_${c}_${sl}.log; exit 1; }
  python - "gpurun_out/cb_${c}_${sl}.log" "$c" "$sl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("chain", sys.argv[2], "slots", sys.argv[3], "ms", round(d["ms_per_step"], 4), "kern_us",
      d["roofline"]["avg_launch_us"], "ticks", d["config"]["schedule_ticks"], "nwg",
      d["config"]["nwg"], "kernel", d["roofline"]["kernel"])
PY
done
