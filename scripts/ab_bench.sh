#!/bin/bash
# A/B of library builds on one GPU box: bash scripts/ab_bench.sh "old new" "448 384"
# (libraries: tx-fast-hydrology_amd/tx_fast_hydrology_amd/lib/exp/lib_<name>.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
E=tx-fast-hydrology_amd/tx_fast_hydrology_amd/lib/exp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in ${1:-old new}; do
    for s in ${2:-448}; do
      MCROUTE_LIB=$PWD/$E/lib_$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 \
          --no-cpu --timing-runs 1 --slots $s ${BENCH_ARGS:-} > gpurun_out/ab_${v}_$s.log 2>&1 \
          || { echo "$v $s failed"; tail -3 gpurun_out/ab_${v}_$s.log; exit 1; }
      python - "gpurun_out/ab_${v}_$s.log" "$v" "$s" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "slots", sys.argv[3], "ms", round(d["ms_per_step"], 4), "kern_us", d["roofline"]["avg_launch_us"], "ticks",
      d["config"]["schedule_ticks"], "nwg", d["config"]["nwg"], "kernel", d["roofline"]["kernel"])
PY
    done
  done
done
