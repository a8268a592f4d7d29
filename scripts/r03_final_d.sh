# Round-3 evidence on the masked-store build, part B (as r03_final_b.sh): rocprofv3 kernel-trace
# summaries of the bench workloads, PMC HBM
# traffic of the routing kernels (FETCH_SIZE and WRITE_SIZE in separate passes, stamped with the
# library's source hash by scripts/hbm_traffic.py), the bench lines that report it, the det
# kernel's SQ counters and the EnKF256 MFMA counters.  Outputs gpurun_out/r03w_*.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
stats() {   # name, bench args
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/r03w_prof_$name" \
      -o run -- python3 "$PWD/bench.py" --no-cpu --no-api --timing-runs 1 "$@" > $O/r03w_prof_$name.log 2>&1
  local rc=$?
  echo "stats $name rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $O/r03w_prof_$name.log; exit $rc; }
  return 0
}
pmc() {   # name, counters, bench args
  local name=$1 ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$PWD/$O/r03w_pmc_$name" \
      -o run -- python3 "$PWD/bench.py" --no-cpu --no-api --timing-runs 1 --steps 1 --warmup 0 "$@" > $O/r03w_pmc_$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $O/r03w_pmc_$name.log; exit $rc; }
  return 0
}
stats det --steps 5 --warmup 1
stats ens64 --steps 2 --warmup 1 --members 64
stats enkf32 --steps 1 --warmup 1 --members 32 --enkf
stats enkf256 --steps 1 --warmup 1 --members 256 --enkf
pmc det_fetch FETCH_SIZE
pmc det_write WRITE_SIZE
pmc ens64_fetch FETCH_SIZE --members 64
pmc ens64_write WRITE_SIZE --members 64
pmc conus_fetch FETCH_SIZE --conus
pmc conus_write WRITE_SIZE --conus
python scripts/hbm_traffic.py $O/r03w_pmc_det_fetch $O/r03w_pmc_det_write r03w 192 16 190000 288 > $O/r03w_traffic.log 2>&1 && \
python scripts/hbm_traffic.py $O/r03w_pmc_ens64_fetch $O/r03w_pmc_ens64_write r03w 256 64 190000 288 64 >> $O/r03w_traffic.log 2>&1 && \
python scripts/hbm_traffic.py $O/r03w_pmc_conus_fetch $O/r03w_pmc_conus_write r03w 256 64 2700000 288 16 >> $O/r03w_traffic.log 2>&1
rc=$?; echo "traffic rc=$rc"; [ $rc -ne 0 ] && { cat $O/r03w_traffic.log; exit $rc; }
mkdir -p $O/r03w_profiles && cp profiles/r03w_hbm_traffic*.json $O/r03w_profiles/
# bench lines that now find a PMC profile of this build
for W in det ens64 conus; do
  A=""; [ $W = ens64 ] && A="--members 64"; [ $W = conus ] && A="--conus"
  timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu $A > $O/r03w_bench_${W}_dram.json 2>&1
  rc=$?; echo "bench ${W}_dram rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/r03w_bench_${W}_dram.json; exit $rc; }
done
pmc det_sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
pmc det_sq2 "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
pmc det_sq3 "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM"
pmc enkf256_mfma "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE" --members 256 --enkf
exit 0
