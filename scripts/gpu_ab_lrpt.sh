#!/bin/bash
# Mixed-batch placement and priority: cur (ranked blocks + longest-remaining-first priority
# for mixed batches), base (HEAD), m1 (ranked blocks, younger-wave priority), norank (priority
# only): GPU parity, interleaved A/B of configs 5, 3 and 2, then the timeline probe.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
AB_TAG=c5 VARIANTS="cur base m1 norank" ROUNDS=3 BENCH_ARGS="--config 5 --pipeline 1" bash scripts/gpu_ab_lib.sh || exit 1
VARIANTS="cur base" ROUNDS=2 BENCH_ARGS="--pipeline 1" bash scripts/gpu_ab_lib.sh || exit 1
AB_TAG=c2 VARIANTS="cur base" ROUNDS=2 BENCH_ARGS="--config 2" bash scripts/gpu_ab_lib.sh || exit 1
timeout -k 10 300 python scripts/exp/vit_trace.py > gpurun_out/vtrace.log 2>&1; rc=$?; cut -c1-300 gpurun_out/vtrace.log; exit $rc
