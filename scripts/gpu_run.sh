#!/bin/bash
# One parameterised GPU-box session (replaces the round-3 one-off scripts/r03_gpu*.sh).
#
#   scripts/gpu_run.sh TAG STEP [STEP ...]
#
# Every step runs under its own time limit, writes its output under gpurun_out/TAG/, and the run
# stops at the first failing step (no retries, nothing more on the GPU after a fault/timeout).
# Steps (KIND:ARGS):
#   pytest:ARGS      python -m pytest -m gpu -x -v ARGS           -> N.pytest.txt
#   bench:ARGS       python bench.py ARGS (one JSON line)         -> N.bench.json
#   stats:NAME:ARGS  rocprofv3 --kernel-trace --stats of bench.py ARGS -> prof_NAME/
#   pmc:NAME:CTRS:ARGS  rocprofv3 --pmc CTRS (one pass) of bench.py ARGS -> pmc_NAME/
#   py:ARGS          python ARGS (a script under scripts/)        -> N.py.txt
#   smoke:           __graft_entry__.smoke()                      -> N.smoke.txt
# Limits: T_PYTEST (900 s), T_STEP (600 s).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
T_PYTEST=${T_PYTEST:-900}
T_STEP=${T_STEP:-600}
i=0
for step in "$@"; do
    i=$((i + 1))
    kind=${step%%:*}
    args=${step#*:}
    case $kind in
    pytest)
        f=$OUT/$i.pytest.txt
        timeout -k 10 "$T_PYTEST" python -u -m pytest -m gpu -x -v --timeout 400 \
            --timeout-method thread -p no:cacheprovider $args > "$f" 2>&1 ;;
    bench)
        f=$OUT/$i.bench.json
        timeout -k 10 "$T_STEP" python -u bench.py $args > "$f" 2> "$OUT/$i.bench.err" ;;
    stats)
        name=${args%%:*}
        f=$OUT/$i.stats.log
        timeout -k 10 "$T_STEP" rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof_$name" \
            -o run --output-format csv -- python3 "$PWD/bench.py" ${args#*:} > "$f" 2>&1 ;;
    pmc)
        name=${args%%:*}
        rest=${args#*:}
        ctrs=${rest%%:*}
        f=$OUT/$i.pmc.log
        timeout -s KILL "$T_STEP" rocprofv3 --pmc $ctrs -d "$PWD/$OUT/pmc_$name" -o run \
            --output-format csv -- python3 "$PWD/bench.py" ${rest#*:} > "$f" 2>&1 ;;
    py)
        f=$OUT/$i.py.txt
        timeout -k 10 "$T_STEP" python -u $args > "$f" 2>&1 ;;
    smoke)
        f=$OUT/$i.smoke.txt
        timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$f" 2>&1 ;;
    *)
        echo "unknown step kind: $kind" >&2
        exit 2 ;;
    esac
    rc=$?
    echo "== step $i ($kind) rc=$rc"
    tail -n 4 "$f"
    if [ $rc -ne 0 ]; then
        exit $rc
    fi
done
