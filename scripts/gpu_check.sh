#!/bin/bash
# GPU session script: parity tests, smoke, short bench.  Stops at the first crash/timeout;
# plain test failures (exit 1) do not stop the later steps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 400 python bench.py --steps ${STEPS:-5} --warmup 2 > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
