#!/bin/bash
# Round 4: A/B of the working tree (cur) against HEAD (prev, scripts/build_variant.sh HEAD prev) after the GPU parity suite
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
VARIANTS="cur prev" ROUNDS=3 STEPS=20 AB_TAG=c3 bash scripts/gpu_ab_lib.sh || exit 1
VARIANTS="cur prev" ROUNDS=2 STEPS=20 AB_TAG=c2 BENCH_ARGS="--config 2" bash scripts/gpu_ab_lib.sh || exit 1
VARIANTS="cur prev" ROUNDS=2 STEPS=10 AB_TAG=c5 BENCH_ARGS="--config 5 --cpu-seconds 0.5" bash scripts/gpu_ab_lib.sh || exit 1
echo r04e-ok
