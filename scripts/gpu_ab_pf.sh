#!/bin/bash
# A/B of the soft prefetch distance (libziria_rx.pf2.so) and the 8-lane DBG attribution sweep (exp).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="cur pf2 v16" ROUNDS=2 BENCH_ARGS="--pipeline 1" bash scripts/gpu_ab_lib.sh || exit 1
LIBV=exp DBGS="0 1 2 4 8 1024 0" BENCH_ARGS="--pipeline 1" bash scripts/gpu_dbg_sweep.sh || exit 1
