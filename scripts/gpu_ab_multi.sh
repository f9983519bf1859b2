#!/bin/bash
# Parity suite, then interleaved A/B of VARIANTS on each workload in CONFIGS (bench.py
# --config N; 3 = default), ROUNDS rounds each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for cfg in ${CONFIGS:-3}; do
  echo "== config $cfg"
  AB_TAG=c$cfg BENCH_ARGS="--config $cfg" VARIANTS="${VARIANTS:-cur}" ROUNDS=${ROUNDS:-2} ./scripts/gpu_ab_lib.sh || exit 1
done
