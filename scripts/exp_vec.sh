#!/bin/bash
# Diagnostic: member-vector kernel variants with one part of the tick removed (MCR_VEXP_*
# switches in vector.hip), timed on one ensemble bench line each.
#     bash scripts/exp_vec.sh build          (here, no GPU needed)
#     bash scripts/exp_vec.sh run "c:t:E:H:W"   (GPU box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PKG=tx-fast-hydrology_amd
OUT=$PKG/tx_fast_hydrology_amd/lib/vexp
VARIANTS="${VARIANTS:-base:-DMCR_VEXP_NONE nostores:-DMCR_VEXP_NO_STORES=1 noloads:-DMCR_VEXP_NO_LOADS=1 nobarrier:-DMCR_VEXP_NO_BARRIER=1}"
if [ "${1:-run}" = build ]; then
  mkdir -p $OUT
  for v in $VARIANTS; do
    name=${v%%:*}; flags=${v#*:}
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
      -fno-fast-math -Iinclude -I$PKG/csrc ${flags//,/ } -o $OUT/lib_$name.so $PKG/csrc/*.cpp \
      $PKG/csrc/*.hip -L/opt/rocm/lib -lrocsolver -lrocblas -Wl,-rpath,/opt/rocm/lib &
  done
  wait
  ls -la $OUT
  exit 0
fi
mkdir -p gpurun_out
IFS=: read c t E H W <<< "${2:-1:32:64:2:16}"
for v in $VARIANTS; do
  name=${v%%:*}
  MCROUTE_LIB=$PWD/$OUT/lib_$name.so timeout -k 10 200 \
      python bench.py --steps 5 --warmup 2 --no-cpu --timing-runs 2 --slots 64 --chain $c \
      --tile $t --members $E --vec-shape ${H:-0}:${W:-0} > gpurun_out/vexp_$name.log 2>&1
  rc=$?
  [ $rc -ne 0 ] && { echo "$name rc=$rc"; tail -5 gpurun_out/vexp_$name.log; exit $rc; }
  python - gpurun_out/vexp_$name.log "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "ms", round(d["ms_per_step"], 3), "kern_ms", d["roofline"]["kernel_ms_per_step"])
PY
done
