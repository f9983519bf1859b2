#!/bin/bash
# Priority-schedule fine tuning: parity on the in-tree build, interleaved A/B of config 3 and
# config 2, then the Viterbi timeline probe (vtrace build) of configs 5 and 3.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="cur p35 p58 p710 p00" ROUNDS=2 BENCH_ARGS="--pipeline 1" bash scripts/gpu_ab_lib.sh || exit 1
AB_TAG=c2 VARIANTS="cur p58 p710" ROUNDS=2 BENCH_ARGS="--config 2" bash scripts/gpu_ab_lib.sh || exit 1
timeout -k 10 300 python scripts/exp/vit_trace.py > gpurun_out/vtrace.log 2>&1; rc=$?; cut -c1-300 gpurun_out/vtrace.log; exit $rc
