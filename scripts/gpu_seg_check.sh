#!/bin/bash
# Segment work loop: GPU parity suite, default / config 2 / config 5 benches, and a rocprof
# kernel trace of config 3 and config 5 (k_pkt_plan, both k_viterbi3 passes).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for a in "" "--config 2" "--config 5"; do
  f=gpurun_out/bench_$(echo "c3 $a" | tr -d ' -').log
  timeout -k 10 200 python bench.py --no-cpu --steps 20 $a > $f 2>&1 || { tail -5 $f; exit 1; }
  python - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(d["config"]["workload"][:40], d["value"], d["ms_per_step"], d.get("stage_ms"))
PY
done
for a in "" "--config 5"; do
  d=gpurun_out/prof_$(echo "c3 $a" | tr -d ' -')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python bench.py --no-cpu --steps 10 --warmup 2 $a > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  python - $d <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "zrx" in r["Name"]:
            print("  ", r["Name"][:48], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
