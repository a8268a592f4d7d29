# SQ counters of the ensemble multi-launch kernel (ens64)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$PWD/$O/r03n_ens_sq$i" -o run -- python3 "$PWD/bench.py" --steps 1 --warmup 0 --no-cpu --timing-runs 1 --members 64 > $O/r03n_ens_sq$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/r03n_ens_sq$i.log; exit $rc; }
done
exit 0
