#!/bin/bash
# Same-box comparison of ensemble / EnKF bench workloads at several session shapes.
# Usage: bash scripts/enkf_cmp.sh "<bench args>" ["<bench args>" ...]
set -u
mkdir -p gpurun_out
for args in "$@"; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --timing-runs 1 $args > gpurun_out/cmp.log 2>&1
  rc=$?
  echo "$args rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/cmp.log; exit $rc; }
  python -c "
import json,sys
l=[x for x in open('gpurun_out/cmp.log') if x.startswith('{')][-1]; d=json.loads(l)
print(' ms/step %.2f value %.3e kernel_ms/step %s launches/step %s' % (d['ms_per_step'], d['value'], d['roofline']['kernel_ms_per_step'], d['roofline']['launches_per_step']))"
done
