#!/bin/bash
# rocprofv3 evidence for bench.py's dominant kernels: kernel-trace stats of the default
# bench command, then separate --pmc passes (SQ/GRBM for VALU issue, FETCH_SIZE, WRITE_SIZE)
# and L1/L2/TA/LDS-conflict counters on the same workload with one timed step.  Summaries -> gpurun_out/ (copy to profiles/).
# --pipeline 1 (one engine): its kernel durations are the ones the bench's roofline uses (the
# instrumented engine-0-alone pass); with two engines in flight rocprof also times overlap.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --no-sub ${BENCH_ARGS:---pipeline 1} > $R/gpurun_out/prof_bench.log 2>&1; rc=$?
echo "rocprof stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE" \
         "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmc$i -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu --no-sub --pipeline 1 ${PMC_ARGS:-} > $R/gpurun_out/pmc$i.log 2>&1; rc=$?
  echo "pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd $R && python scripts/pmc_summary.py gpurun_out > gpurun_out/pmc_summary.json; echo "summary rc=$?"
