#!/bin/bash
# Mixed-batch segment length with the ranked placement: cur (11/8 L) against 6/8, 8/8, 9/8
# and the longest-remaining-first priority build (m3), interleaved on config 5.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_TAG=c5 VARIANTS="cur mix6 mix8 mix9 m3" ROUNDS=3 BENCH_ARGS="--config 5 --pipeline 1" bash scripts/gpu_ab_lib.sh || exit 1
for v in mix6 mix8 mix9; do
  ZRX_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_segments.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1; rc=$?
  echo "$v parity rc=$rc"; tail -1 gpurun_out/pytest_$v.log; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
done
