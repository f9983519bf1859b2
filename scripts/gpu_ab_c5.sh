#!/bin/bash
# Interleaved A/B of config 5 (VARIANTS) with the pipelined default bench settings.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_TAG=c5 VARIANTS="$VARIANTS" ROUNDS=${ROUNDS:-2} BENCH_ARGS="--config 5" bash scripts/gpu_ab_lib.sh
