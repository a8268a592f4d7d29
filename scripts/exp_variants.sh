#!/bin/bash
# Diagnostic: build kernel variants with one part of the tick removed (MCR_EXP_* switches in
# kernels.hip) and trace one bench horizon with each.  Build here (no GPU needed):
#     bash scripts/exp_variants.sh build
# and run on the GPU box:
#     bash scripts/exp_variants.sh run
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PKG=tx-fast-hydrology_amd
OUT=$PKG/tx_fast_hydrology_amd/lib/exp
VARIANTS="${VARIANTS:-base:-DMCR_EXP_NONE nostores:-DMCR_EXP_NO_STORES=1 nobarrier:-DMCR_EXP_NO_BARRIER=1 noq:-DMCR_EXP_NO_Q=1} ${EXTRA_VARIANTS:-}"
if [ "${1:-run}" = build ]; then
  mkdir -p $OUT
  for v in $VARIANTS; do
    name=${v%%:*}; flags=${v#*:}
    python $PKG/tx_fast_hydrology_amd/_build.py --variant $name ${flags//,/ } > /dev/null &
  done
  wait
  ls -la $OUT
  exit 0
fi
mkdir -p gpurun_out
for v in $VARIANTS; do
  name=${v%%:*}
  MCROUTE_LIB=$PWD/$OUT/lib_$name.so timeout -k 10 200 python scripts/trace_launches.py \
      "exp_$name" --quiet ${TRACE_ARGS:-} > gpurun_out/exp_$name.log 2>&1
  rc=$?
  grep SUMMARY gpurun_out/exp_$name.log | sed "s/^/$name /"
  [ $rc -ne 0 ] && { echo "$name rc=$rc"; tail -5 gpurun_out/exp_$name.log; exit $rc; }
done
exit 0
