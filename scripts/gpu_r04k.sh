#!/bin/bash
# Round 4: config 5 with the dynamic task queue: mixed cut length (11/8, 8/8, 6/8 L) and the
# younger-wave priority (np: off), against the static placement (cur); interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
VARIANTS="cur dyn11np dyn8 dyn8np dyn6" ROUNDS=2 STEPS=10 AB_TAG=k5 BENCH_ARGS="--config 5 --cpu-seconds 0.2" bash scripts/gpu_ab_lib.sh || exit 1
VARIANTS="dyn8 dyn8np dyn6 cur" ROUNDS=1 STEPS=10 AB_TAG=k5p1 BENCH_ARGS="--config 5 --pipeline 1 --cpu-seconds 0.2" bash scripts/gpu_ab_lib.sh || exit 1
echo r04k-ok
