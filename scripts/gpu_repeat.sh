#!/bin/bash
# The workspace event without a system-scope fence (cur), recorded only when a launch changes
# streams (lazy), against the previous commit (prev); configs 3 and 5 and a 2048-packet shard.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
VARIANTS="cur prev lazy" ROUNDS=3 STEPS=20 AB_TAG=r3 bash scripts/gpu_ab_lib.sh || exit 1
VARIANTS="cur prev lazy" ROUNDS=2 STEPS=40 AB_TAG=r2k BENCH_ARGS="--npkts 2048" bash scripts/gpu_ab_lib.sh || exit 1
VARIANTS="cur prev lazy" ROUNDS=1 STEPS=10 AB_TAG=r5 BENCH_ARGS="--config 5 --cpu-seconds 0.2" bash scripts/gpu_ab_lib.sh || exit 1
