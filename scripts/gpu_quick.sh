#!/bin/bash
# Short GPU session: the parity suite, interleaved A/B of VARIANTS on the default bench
# (ROUNDS), and a rocprof kernel trace of the in-tree build (config 3).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
VARIANTS="${VARIANTS:-cur}" ROUNDS=${ROUNDS:-3} ./scripts/gpu_ab_lib.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof_c3.log 2>&1 || { tail -5 gpurun_out/prof_c3.log; exit 1; }
python - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof_c3/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "zrx" in r["Name"]:
            print(r["Name"][:44], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), r["MinNs"], r["MaxNs"])
PY
