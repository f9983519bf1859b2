#!/bin/bash
# parity tests, bench, kernel-trace stats and one PMC pass on the Viterbi kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; ok $rc || exit $rc
python - <<'PY'
import json
for l in open("gpurun_out/bench.log"):
    if l.startswith("{"):
        d = json.loads(l); print(d["value"], d["ms_per_step"], d["stage_ms"], d["roofline"]["frac"], d["bit_exact_check"])
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu > $R/gpurun_out/prof.log 2>&1; rc=$?
echo "rocprof stats rc=$rc"; ok $rc || exit $rc
if [ -n "$PMC" ]; then
  timeout -k 10 300 rocprofv3 --pmc $PMC --output-format csv -d $R/gpurun_out/pmc -o pmc -- python3 $R/bench.py --npkts 4096 --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/pmc.log 2>&1; rc=$?
  echo "rocprof pmc rc=$rc"
fi
exit 0
