#!/bin/bash
# Parity suite, then interleaved A/B of VARIANTS over several workloads (ARGSETS, separated by
# ';'), ROUNDS rounds each: prints the data-Viterbi stage, ms/step and Gbit/s per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
fi
IFS=';' read -ra SETS <<< "${ARGSETS:-}"
i=0
for a in "${SETS[@]}"; do
  echo "== $a"
  AB_TAG=s$i BENCH_ARGS="$a" ./scripts/gpu_ab_lib.sh || exit 1
  i=$((i+1))
done
