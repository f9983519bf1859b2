#!/bin/bash
# Config 5: more than two block rounds with the blocks in plain longest-first dispatch order (the
# ZRX_RANK_LPT switch of commit "rank_place: ZRX_RANK_LPT A/B switch", since removed: re-add it to rerun)
# (ZRX_RANK_LPT) at segment cuts of 8/8, 9/8, 10/8, 11/8 L, against the in-tree build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_TAG=c5 VARIANTS="cur lpt8 lpt9 lpt10 lpt11" ROUNDS=3 BENCH_ARGS="--config 5 --pipeline 1" bash scripts/gpu_ab_lib.sh || exit 1
for v in lpt8 lpt9; do
  ZRX_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1; rc=$?
  echo "$v parity rc=$rc"; tail -1 gpurun_out/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
