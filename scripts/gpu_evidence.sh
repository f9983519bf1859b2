#!/bin/bash
# Evidence run: GPU parity suite, smoke, the driver's bench command, rocprof kernel
# stats + PMC passes (scripts/gpu_pmc.sh), the config-4 strong-scaling shard sizes, the other
# BASELINE configs and §8f rows, the host-sanitized driver's GPU tests, the per-call bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-160
bash scripts/gpu_pmc.sh || exit 1
for n in 2048 4096 8192; do
  timeout -k 10 300 python bench.py --npkts $n --steps 40 --warmup 5 --no-cpu > gpurun_out/bench_n$n.log 2>&1 || { tail -5 gpurun_out/bench_n$n.log; exit 1; }
  tail -1 gpurun_out/bench_n$n.log | cut -c1-120
done
for a in "--config 1" "--config 2" "--config 5 --steps 40" "--eq" "--tx"; do
  f=gpurun_out/bench_$(echo $a | tr -d ' -').log
  timeout -k 10 300 python bench.py --steps 10 $a > $f 2>&1 || { echo "bench $a failed"; tail -5 $f; exit 1; }
  tail -1 $f | cut -c1-140
done
cd /tmp && export TMPDIR=/tmp && R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5 -o run -- python3 $R/bench.py --config 5 --steps 5 --warmup 2 --cpu-seconds 1 > $R/gpurun_out/prof_c5.log 2>&1 || { tail -5 $R/gpurun_out/prof_c5.log; exit 1; }
cd $R
ZRX_DRIVER=ziria_amd/_lib/asan/ziria_rx_driver ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  timeout -k 10 300 python -u -m pytest tests/test_driver.py -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/asan_driver.log 2>&1 || { tail -5 gpurun_out/asan_driver.log; exit 1; }
tail -1 gpurun_out/asan_driver.log
timeout -k 10 120 ziria_amd/_lib/percall_bench 10 1500 > gpurun_out/percall.json 2>&1 || exit 1
echo evidence-ok
