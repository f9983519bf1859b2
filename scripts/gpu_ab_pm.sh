#!/bin/bash
# Config 5 with the ranked placement: the younger-wave priority (in-tree) against none for
# (pm0 was built with a ZRX_PRIO_MIXED=0 switch, since removed; m0 = -DZRX_PRIO_MODE=0)
# mixed batches (pm0) and none at all (m0).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_TAG=c5 VARIANTS="cur pm0 m0" ROUNDS=4 BENCH_ARGS="--config 5 --pipeline 1" bash scripts/gpu_ab_lib.sh || exit 1
ZRX_LIB_VARIANT=pm0 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pm0.log 2>&1; rc=$?
echo "pm0 parity rc=$rc"; tail -1 gpurun_out/pytest_pm0.log; exit $rc
