#!/bin/bash
# Same-box A/B of library builds (lib/exp/lib_<name>.so, scripts/mkvar.sh), one bench line each,
# REPS rounds in alternating order:
#     REPS=2 BENCH_ARGS="--members 64" bash scripts/ab.sh TAG "base new"
# prints one summary line per run; logs under gpurun_out/<TAG>_<name>_<rep>.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1
VARIANTS=$2
E=tx-fast-hydrology_amd/tx_fast_hydrology_amd/lib/exp
mkdir -p gpurun_out
for rep in $(seq 1 "${REPS:-2}"); do
  for v in $VARIANTS; do
    lib=$PWD/$E/lib_$v.so
    [ "$v" = "main" ] && lib=$PWD/tx-fast-hydrology_amd/tx_fast_hydrology_amd/lib/libmcroute.so
    log=gpurun_out/${TAG}_${v}_${rep}.log
    MCROUTE_LIB=$lib timeout -k 10 ${TLIM:-240} python bench.py --steps ${STEPS:-20} --warmup 3 \
        --no-cpu --no-api --timing-runs 1 ${BENCH_ARGS:-} > "$log" 2>&1 \
        || { echo "$v rep $rep failed"; tail -5 "$log"; exit 1; }
    python - "$log" "$v" "$rep" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
print(sys.argv[2], "rep", sys.argv[3], "ms", round(d["ms_per_step"], 4),
      "kern_us", r.get("avg_launch_us"), "ticks", d["config"].get("schedule_ticks"),
      "nwg", d["config"].get("nwg"), "kernel", r.get("kernel"))
PY
  done
done
