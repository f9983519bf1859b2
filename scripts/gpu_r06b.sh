#!/bin/bash
# Parity suite, the default bench line, and rocprof kernel traces of the headline and config 5.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r06b}
echo "== pytest $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench $(date +%T)"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 15 > gpurun_out/${T}_bench.log 2>&1; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_bench.log; exit $rc; }
echo "== rocprof headline $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c3 -o run -- python bench.py --steps 20 --warmup 15 --no-cpu --no-sub > gpurun_out/${T}_prof_c3.log 2>&1; rc=$?
echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_prof_c3.log; exit $rc; }
echo "== rocprof config5 $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c5 -o run -- python bench.py --config 5 --steps 20 --warmup 15 --cpu-seconds 0.1 > gpurun_out/${T}_prof_c5.log 2>&1; rc=$?
echo "rocprof c5 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_prof_c5.log; exit $rc; }
exit 0
