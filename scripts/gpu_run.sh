#!/bin/bash
# GPU session: parity tests, then (only if they pass) the bench for each Viterbi impl in
# $IMPLS (default "3 2"), then a rocprofv3 kernel-trace of the default bench.
# Every GPU step has its own time limit; the script stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ -n "$BENCH_ANYWAY" ] || exit $rc
for v in ${IMPLS:-3 2}; do
  ZRX_VITERBI=$v timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu > gpurun_out/bench_v$v.log 2>&1; rc=$?
  echo "bench v$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python - "$v" <<'PY'
import json, sys
for l in open(f"gpurun_out/bench_v{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l); print("v" + sys.argv[1], d["value"], d["ms_per_step"], d["stage_ms"], d["roofline"]["frac"], d["bit_exact_check"])
PY
done
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu > $R/gpurun_out/prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"; exit $rc
fi
exit 0
