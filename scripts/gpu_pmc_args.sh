#!/bin/bash
# rocprofv3 kernel trace + PMC passes of one bench.py workload (BENCH_ARGS, e.g. "--eq"), into
# gpurun_out/$OUT/{prof,pmc1..pmc5}; summarise with
#   python scripts/pmc_summary.py gpurun_out/$OUT
# (pass 4: cache/TA/LDS counters; pass 5: where the address path stalls).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=${OUT:-pmcargs}
mkdir -p gpurun_out/$OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$OUT/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --pipeline 1 ${BENCH_ARGS:-} > $R/gpurun_out/$OUT/prof_bench.log 2>&1; rc=$?
echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE" \
         "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM" \
         "SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/$OUT/pmc$i -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu --pipeline 1 ${BENCH_ARGS:-} > $R/gpurun_out/$OUT/pmc$i.log 2>&1; rc=$?
  echo "pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
