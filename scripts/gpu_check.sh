#!/bin/bash
# GPU session: parity tests, then (only if they pass) the default bench line.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ls oracle > gpurun_out/snapshot_oracle_ls.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | cut -c1-1500
exit $rc
