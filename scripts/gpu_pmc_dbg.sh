#!/bin/bash
# PMC instruction counts of k_viterbi3 under ZRX_V3DBG timing variants (experiments build
# libziria_rx.exp.so): where the non-column overhead goes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for d in 0 1; do
  ZRX_LIB_VARIANT=exp ZRX_V3DBG=$d timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmcdbg$d -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu --pipeline 1 > $R/gpurun_out/pmcdbg$d.log 2>&1; rc=$?
  echo "dbg $d rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
