#!/bin/bash
# Round-6 GPU session: the parity suite (with the node / host-register tests), then the
# default bench line (headline + sub-results), then the end-to-end drop-in bench.  Every step
# has its own time limit; the first failure ends the session.  TAG names the output files.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r06}
step() { echo "== $1 $(date +%T)"; }
if [ -z "$SKIP_PYTEST" ]; then
  step pytest
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
    > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$AB" ]; then
  step ab
  VARIANTS="$AB" ROUNDS=${ROUNDS:-3} STEPS=${STEPS:-20} ./scripts/gpu_ab_lib.sh > gpurun_out/${T}_ab.txt 2>&1; rc=$?
  cat gpurun_out/${T}_ab.txt
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$AB_EQ" ]; then
  step ab-eq
  VARIANTS="$AB_EQ" AB_TAG=eq ROUNDS=${ROUNDS:-3} STEPS=${STEPS:-20} BENCH_ARGS="--eq" ./scripts/gpu_ab_lib.sh > gpurun_out/${T}_ab_eq.txt 2>&1; rc=$?
  cat gpurun_out/${T}_ab_eq.txt
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$SKIP_BENCH" ]; then
  step bench
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 15} > gpurun_out/${T}_bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -1 gpurun_out/${T}_bench.log | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$E2E" ]; then
  step e2e
  timeout -k 10 300 python -u bench.py --e2e --steps 10 --warmup 3 > gpurun_out/${T}_e2e.log 2>&1; rc=$?
  echo "e2e rc=$rc"; tail -1 gpurun_out/${T}_e2e.log | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
