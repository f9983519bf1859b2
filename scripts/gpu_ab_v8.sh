#!/bin/bash
# 8-lane Viterbi rows: GPU parity suite, then interleaved A/B of configs 3, 2 and 5 against
# the 16-lane build (libziria_rx.v16.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
VARIANTS="cur v16" ROUNDS=2 BENCH_ARGS="--pipeline 1" bash scripts/gpu_ab_lib.sh || exit 1
AB_TAG=c2 VARIANTS="cur v16" ROUNDS=2 BENCH_ARGS="--config 2" bash scripts/gpu_ab_lib.sh || exit 1
AB_TAG=c5 VARIANTS="cur v16" ROUNDS=2 BENCH_ARGS="--config 5" bash scripts/gpu_ab_lib.sh || exit 1
