#!/bin/bash
# Per-kernel A/B of library builds (lib/exp/lib_<name>.so), same box: one rocprofv3
# --kernel-trace --stats run of bench.py per variant, the kernels matching PATTERN summarised.
#     bash scripts/ab_stats.sh "a b c" "<bench args>" "pattern|pattern"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
E=tx-fast-hydrology_amd/tx_fast_hydrology_amd/lib/exp
mkdir -p gpurun_out/abs
for v in $1; do
  MCROUTE_LIB=$PWD/$E/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      -d "$PWD/gpurun_out/abs/$v" -o run --output-format csv -- \
      python3 "$PWD/bench.py" --no-cpu --timing-runs 1 $2 > gpurun_out/abs/$v.log 2>&1 \
      || { echo "$v failed"; tail -5 gpurun_out/abs/$v.log; exit 1; }
  python3 - "gpurun_out/abs/$v" "$v" "$3" <<'PY'
import csv, glob, json, re, sys
d, name, pat = sys.argv[1], sys.argv[2], sys.argv[3]
f = glob.glob(d + "/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
out = [f"{name}: total {tot / 1e6:.2f} ms"]
for r in rows:
    if re.search(pat, r["Name"]):
        out.append(f"  {r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1e3:8.1f} us")
print("\n".join(out))
PY
done
