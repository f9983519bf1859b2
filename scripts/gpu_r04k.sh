#!/bin/bash
# Round 4: SIGNAL Viterbi on 8-lane rows -- GPU parity suite, then interleaved A/B against the
# previous commit (prev: one wave per packet) on configs 3 and 5; config 5 with the dynamic
# task queue: mixed cut length (11/8, 8/8, 6/8 L) and the younger-wave priority (np: off);
# config 3 with the soft fetch two bodies ahead (vpf2).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
VARIANTS="cur prev vpf2" ROUNDS=3 STEPS=20 AB_TAG=k3 bash scripts/gpu_ab_lib.sh || exit 1
VARIANTS="cur prev dyn11np dyn8 dyn8np dyn6" ROUNDS=2 STEPS=10 AB_TAG=k5 BENCH_ARGS="--config 5 --cpu-seconds 0.2" bash scripts/gpu_ab_lib.sh || exit 1
echo r04k-ok
