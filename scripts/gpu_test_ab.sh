#!/bin/bash
# GPU session: parity tests (PYTEST_K selects), then, if green, interleaved A/B timing of
# engine builds (scripts/gpu_ab_lib.sh: VARIANTS, ROUNDS, STEPS, BENCH_ARGS).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
./scripts/gpu_ab_lib.sh
