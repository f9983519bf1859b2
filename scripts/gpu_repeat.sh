#!/bin/bash
# descramble/CRC loading the next packet's slot and header while working on this one
# against the previous commit (prev); GPU parity first.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
VARIANTS="cur prev" ROUNDS=3 STEPS=20 AB_TAG=s3 bash scripts/gpu_ab_lib.sh || exit 1
