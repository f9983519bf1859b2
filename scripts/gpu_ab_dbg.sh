#!/bin/bash
# GPU session for a Viterbi column change: full GPU parity suite on the default kernel,
# Viterbi/chain parity on each ZRX_V3DBG variant in $CHECK, then the default bench for each
# variant in $DBGS (ZRX_V3DBG values; 0 = product kernel), interleaved $ROUNDS times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for d in ${CHECK:-}; do
  ZRX_V3DBG=$d timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "viterbi or chain" > gpurun_out/pytest_dbg$d.log 2>&1; rc=$?
  echo "parity dbg=$d rc=$rc"; tail -2 gpurun_out/pytest_dbg$d.log; [ $rc -eq 0 ] || exit $rc
done
for r in $(seq ${ROUNDS:-2}); do
  for d in ${DBGS:-0}; do
    ZRX_V3DBG=$d timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu ${BENCH_ARGS:-} > gpurun_out/abd_${d}_$r.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "dbg $d rc=$rc"; tail -5 gpurun_out/abd_${d}_$r.log; exit $rc; }
    python -c "
import json
for l in open('gpurun_out/abd_${d}_$r.log'):
    if l.startswith('{'): d=json.loads(l); print('dbg ${d}', d.get('stage_ms', {}).get('data_viterbi'), d['ms_per_step'], d['value'], d.get('bit_exact_check'))"
  done
done
