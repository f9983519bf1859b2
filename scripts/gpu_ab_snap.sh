#!/bin/bash
# A/B of the snapshot store forms (libziria_rx.snap1/snap2.so) against the in-tree build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="cur snap1 snap2" ROUNDS=3 BENCH_ARGS="--pipeline 1" bash scripts/gpu_ab_lib.sh || exit 1
AB_TAG=c2 VARIANTS="cur snap1 snap2" ROUNDS=2 BENCH_ARGS="--config 2" bash scripts/gpu_ab_lib.sh || exit 1
