#!/bin/bash
# parity tests + A/B bench of Viterbi v1 vs v2 + rocprof kernel stats of the default bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
[ $rc -eq 0 ] || exit 1
ZRX_VITERBI=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_v1.log 2>&1; rc=$?
echo "bench v1 rc=$rc"; ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_v2.log 2>&1; rc=$?
echo "bench v2 rc=$rc"; ok $rc || exit $rc
python - <<'PY'
import json
for f in ("gpurun_out/bench_v1.log", "gpurun_out/bench_v2.log"):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); print(f, d["value"], d["ms_per_step"], d["stage_ms"], d["roofline"]["frac"], d["bit_exact_check"], d.get("cpu_baseline"))
PY
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof" -o run -- python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --steps 5 --warmup 2 --no-cpu > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof.log" 2>&1; rc=$?
echo "rocprof rc=$rc"
exit $rc
