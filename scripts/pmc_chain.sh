set -u
export TMPDIR=/tmp
for cs in 2:192 3:256; do c=${cs%%:*}; sl=${cs#*:}
BENCH_ARGS="--chain $c --slots $sl" timeout -k 10 250 bash scripts/gpu_pmc.sh k$c "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY" || exit 1
done
timeout -k 10 300 bash scripts/chain_bench.sh "2:192 3:256 4:192"
