#!/bin/bash
# GPU parity suite, then interleaved A/B: config 3 (VARIANTS3), config 5 (VARIANTS5).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
[ -n "$VARIANTS3" ] && { VARIANTS="$VARIANTS3" ROUNDS=${ROUNDS:-2} BENCH_ARGS="--pipeline 1" bash scripts/gpu_ab_lib.sh || exit 1; }
[ -n "$VARIANTS5" ] && { AB_TAG=c5 VARIANTS="$VARIANTS5" ROUNDS=${ROUNDS:-2} BENCH_ARGS="--config 5" bash scripts/gpu_ab_lib.sh || exit 1; }
[ -n "$VARIANTS2" ] && { AB_TAG=c2 VARIANTS="$VARIANTS2" ROUNDS=${ROUNDS:-2} BENCH_ARGS="--config 2" bash scripts/gpu_ab_lib.sh || exit 1; }
exit 0
