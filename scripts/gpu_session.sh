#!/bin/bash
# One GPU session: parity suite, then (if green) interleaved A/B of the default bench against
# the libraries named in VARIANTS, the config-5 bench, its rocprof kernel trace, the
# per-call latency bench and the driver's GPU tests through the host-sanitized build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
step ab
VARIANTS="${VARIANTS:-cur}" ROUNDS=${ROUNDS:-2} ./scripts/gpu_ab_lib.sh || exit 1
step ab-config2
AB_TAG=c2 VARIANTS="${VARIANTS2:-${VARIANTS:-cur}}" ROUNDS=${ROUNDS:-2} BENCH_ARGS="--config 2" ./scripts/gpu_ab_lib.sh || exit 1
step config5
timeout -k 10 300 python bench.py --config 5 --steps 10 > gpurun_out/bench_c5.log 2>&1 || { tail -5 gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log | cut -c1-900
step config5-rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python bench.py --config 5 --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_c5.log 2>&1 || { tail -5 gpurun_out/prof_c5.log; exit 1; }
find gpurun_out/prof_c5 -name "*kernel_stats.csv" | head -1 | xargs -r head -12 | cut -d, -f1-8
step config3-rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof_c3.log 2>&1 || { tail -5 gpurun_out/prof_c3.log; exit 1; }
find gpurun_out/prof_c3 -name "*kernel_stats.csv" | head -1 | xargs -r head -12 | cut -d, -f1-8
step percall
timeout -k 10 120 ziria_amd/_lib/percall_bench 10 1500 > gpurun_out/percall.json 2>&1 || { cat gpurun_out/percall.json; exit 1; }
cat gpurun_out/percall.json
step dbg-config2
LIBV=exp DBGS="${DBGS2:-0 1 2 4 8 16 1024 0}" BENCH_ARGS="--config 2" ./scripts/gpu_dbg_sweep.sh || exit 1
step asan-driver
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 ZRX_DRIVER=ziria_amd/_lib/asan/ziria_rx_driver \
  timeout -k 10 300 python -u -m pytest tests/test_driver.py -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/asan_driver.log 2>&1; rc=$?
echo "asan driver rc=$rc"; tail -4 gpurun_out/asan_driver.log
exit $rc
