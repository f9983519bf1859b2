#!/bin/bash
# descramble/CRC with the slot loads issued with the header loads and the scrambler state
# from the slot's first word (one dependent load less) against the previous commit (prev).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
VARIANTS="cur prev" ROUNDS=3 STEPS=20 AB_TAG=q3 bash scripts/gpu_ab_lib.sh || exit 1
VARIANTS="cur prev" ROUNDS=1 STEPS=10 AB_TAG=q5 BENCH_ARGS="--config 5 --cpu-seconds 0.2" bash scripts/gpu_ab_lib.sh || exit 1
