#!/bin/bash
# Round 4: dynamic LPT task queue for mixed batches + descramble/CRC by buffer ops -- GPU
# parity suite, rocprof kernel stats (configs 3 and 5), A/B against HEAD (prev).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_j3 -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu > $R/gpurun_out/prof_j3.log 2>&1 || { tail -5 $R/gpurun_out/prof_j3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_j5 -o run -- python3 $R/bench.py --config 5 --pipeline 1 --steps 5 --warmup 2 --cpu-seconds 0.2 > $R/gpurun_out/prof_j5.log 2>&1 || { tail -5 $R/gpurun_out/prof_j5.log; exit 1; }
cd $R
for f in prof_j3 prof_j5; do echo "== $f"; python -c "
import csv
for r in csv.DictReader(open('gpurun_out/$f/run_kernel_stats.csv')):
    if 'zrx' in r['Name']: print(r['Name'][:40], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])"; done
VARIANTS="cur prev" ROUNDS=3 STEPS=10 AB_TAG=c5 BENCH_ARGS="--config 5 --cpu-seconds 0.2" bash scripts/gpu_ab_lib.sh || exit 1
VARIANTS="cur prev" ROUNDS=2 STEPS=20 AB_TAG=c3 bash scripts/gpu_ab_lib.sh || exit 1
echo r04j-ok
