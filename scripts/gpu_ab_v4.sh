#!/bin/bash
# 4-lane Viterbi rows (libziria_rx.v4.so): the Viterbi/chain parity tests on the variant, then
# interleaved A/B against the in-tree 8-lane build on configs 3, 2 and 5.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ZRX_LIB_VARIANT=v4 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_v4.log 2>&1; rc=$?
echo "pytest v4 rc=$rc"; tail -2 gpurun_out/pytest_v4.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_v4.log | head; exit $rc; }
VARIANTS="cur v4" ROUNDS=2 BENCH_ARGS="--pipeline 1" bash scripts/gpu_ab_lib.sh || exit 1
AB_TAG=c2 VARIANTS="cur v4" ROUNDS=2 BENCH_ARGS="--config 2" bash scripts/gpu_ab_lib.sh || exit 1
AB_TAG=c5 VARIANTS="cur v4" ROUNDS=2 BENCH_ARGS="--config 5" bash scripts/gpu_ab_lib.sh || exit 1
