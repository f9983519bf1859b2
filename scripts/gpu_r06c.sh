#!/bin/bash
# Parity suite, then interleaved A/B of the current engine against VARIANTS on configs 3 and 5
# and the config-5 kernel trace with one engine (--pipeline 1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r06c}
echo "== pytest $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== ab config 3 $(date +%T)"
VARIANTS="${VARIANTS:-cur prev}" AB_TAG=c3 ROUNDS=${ROUNDS:-3} STEPS=20 ./scripts/gpu_ab_lib.sh > gpurun_out/${T}_ab_c3.txt 2>&1; rc=$?
cat gpurun_out/${T}_ab_c3.txt; [ $rc -eq 0 ] || exit $rc
echo "== ab config 5 $(date +%T)"
VARIANTS="${VARIANTS:-cur prev}" AB_TAG=c5 ROUNDS=${ROUNDS:-3} STEPS=20 BENCH_ARGS="--config 5 --cpu-seconds 0.1" ./scripts/gpu_ab_lib.sh > gpurun_out/${T}_ab_c5.txt 2>&1; rc=$?
cat gpurun_out/${T}_ab_c5.txt; [ $rc -eq 0 ] || exit $rc
echo "== rocprof config5 p1 $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c5p1 -o run -- python bench.py --config 5 --pipeline 1 --steps 20 --warmup 15 --cpu-seconds 0.1 > gpurun_out/${T}_prof_c5p1.log 2>&1; rc=$?
echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_prof_c5p1.log; exit $rc; }
python scripts/kstats.py gpurun_out/${T}_prof_c5p1/run_kernel_stats.csv
exit 0
