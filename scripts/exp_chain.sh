#!/bin/bash
# Diagnostic variants (scripts/exp_variants.sh build) traced at several (chain, slots) shapes:
#     bash scripts/exp_chain.sh "base nohelper" "2:192 3:256"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
E=tx-fast-hydrology_amd/tx_fast_hydrology_amd/lib/exp
for v in ${1:-base}; do
  for cs in ${2:-2:192}; do
    c=${cs%%:*}; sl=${cs#*:}
    MCROUTE_LIB=$PWD/$E/lib_$v.so timeout -k 10 200 python scripts/trace_launches.py \
        "x_${v}_$c" --quiet --chain $c --slots $sl > gpurun_out/x_${v}_$c.log 2>&1 \
        || { echo "$v $cs failed"; tail -3 gpurun_out/x_${v}_$c.log; exit 1; }
    echo "$v chain $c slots $sl: $(grep SUMMARY gpurun_out/x_${v}_$c.log)"
  done
done
