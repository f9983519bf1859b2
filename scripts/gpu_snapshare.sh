#!/bin/bash
# The Viterbi snapshot-store bank conflicts: A/B of the product engine against the timing
# variant whose stores are conflict-free (ZRX_SNAP_SHARE, wrong output by design), then one
# LDS-counter pass of each (bank-conflict cycles, LDS instructions, LDS-array cycles).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
VARIANTS="cur snapshare" ROUNDS=${ROUNDS:-3} STEPS=20 ./scripts/gpu_ab_lib.sh > gpurun_out/snap_ab.txt 2>&1; rc=$?
cat gpurun_out/snap_ab.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp
for v in cur snapshare; do
  if [ "$v" = cur ]; then unset ZRX_LIB_VARIANT; else export ZRX_LIB_VARIANT=$v; fi
  timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES --output-format csv -d $R/gpurun_out/snap_pmc_$v -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu --no-sub --pipeline 1 > $R/gpurun_out/snap_pmc_$v.log 2>&1; rc=$?
  echo "pmc $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
