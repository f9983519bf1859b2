#!/bin/bash
# Round 4: the SIGNAL decode fused into one kernel (k_signal: FFT in wave 0, rows in all 8)
# against the previous commit (prev: k_signal_fft + k_signal_vit); configs 3 and 5.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
VARIANTS="cur prev" ROUNDS=3 STEPS=20 AB_TAG=o3 bash scripts/gpu_ab_lib.sh || exit 1
VARIANTS="cur prev" ROUNDS=1 STEPS=10 AB_TAG=o5 BENCH_ARGS="--config 5 --cpu-seconds 0.2" bash scripts/gpu_ab_lib.sh || exit 1
echo r04o-ok
