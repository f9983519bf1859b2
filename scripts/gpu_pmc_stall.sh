#!/bin/bash
# Stall attribution PMC passes for the default bench (one engine): where waves wait.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
i=10
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT" \
         "SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmc$i -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu --pipeline 1 > $R/gpurun_out/pmc$i.log 2>&1; rc=$?
  echo "pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
