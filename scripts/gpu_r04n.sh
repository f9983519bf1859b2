#!/bin/bash
# Round 4: k_data_fft locating the next wave's symbols (scalar boundary loads, parameter loads
# issued) under the current wave's FFT, and descramble/CRC issuing slot, header, chunk and
# received-CRC loads together, against the previous commit (prev).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
VARIANTS="cur prev" ROUNDS=3 STEPS=20 AB_TAG=n3 bash scripts/gpu_ab_lib.sh || exit 1
VARIANTS="cur prev" ROUNDS=1 STEPS=10 AB_TAG=n5 BENCH_ARGS="--config 5 --cpu-seconds 0.2" bash scripts/gpu_ab_lib.sh || exit 1
echo r04n-ok
