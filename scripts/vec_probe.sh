#!/bin/bash
# Member-vector ensemble sweep: GPU parity, then Texas ensemble bench lines at several plan shapes
#     bash scripts/vec_probe.sh "chain:tile:members[:H:waves] ..." [--no-tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${2:-}" != "--no-tests" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
      tests/test_gpu_vector.py > gpurun_out/vec_tests.log 2>&1
  rc=$?; echo "vector tests rc=$rc"; tail -12 gpurun_out/vec_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
for cfg in ${1:-1:32:64}; do
  IFS=: read c t E H W <<< "$cfg"
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --timing-runs 2 --slots 64 \
      --chain $c --tile $t --members $E --vec-shape ${H:-0}:${W:-0} ${BENCH_ARGS:-} > gpurun_out/vb_${c}_${t}_${E}_${H:-0}_${W:-0}.log 2>&1 \
      || { echo "bench $cfg failed"; tail -5 gpurun_out/vb_${c}_${t}_${E}_${H:-0}_${W:-0}.log; exit 1; }
  python - gpurun_out/vb_${c}_${t}_${E}_${H:-0}_${W:-0}.log "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "ms", round(d["ms_per_step"], 3), "value %.3e" % d["value"], "kern_ms",
      r["kernel_ms_per_step"], "launches", r["launches_per_step"], "kernel", r["kernel"],
      "ticks", d["config"]["schedule_ticks"], "nwg", d["config"]["nwg"])
PY
done
