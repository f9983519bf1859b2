#!/bin/bash
# EQ data kernel variant: parity of the variant library on the EQ tests, then interleaved A/B on --eq.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=${V:-eqnostage}
ZRX_LIB_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_eq.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "eq or EQ" > gpurun_out/eqab_pytest_$V.log 2>&1; rc=$?
echo "variant parity rc=$rc"; tail -2 gpurun_out/eqab_pytest_$V.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="cur $V" AB_TAG=eq ROUNDS=${ROUNDS:-3} STEPS=20 BENCH_ARGS="--eq" ./scripts/gpu_ab_lib.sh > gpurun_out/eqab_$V.txt 2>&1; rc=$?
cat gpurun_out/eqab_$V.txt; exit $rc
