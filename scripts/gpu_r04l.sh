#!/bin/bash
# Round 4: descramble/CRC with the next packet prefetched and the slot staged in LDS (cur)
# against the previous commit (prev), and the swizzled demap LUT in k_data_fft (swz).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
VARIANTS="cur prev swz" ROUNDS=3 STEPS=20 AB_TAG=l3 bash scripts/gpu_ab_lib.sh || exit 1
VARIANTS="cur prev swz" ROUNDS=1 STEPS=10 AB_TAG=l5 BENCH_ARGS="--config 5 --cpu-seconds 0.2" bash scripts/gpu_ab_lib.sh || exit 1
echo r04l-ok
