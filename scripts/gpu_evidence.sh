#!/bin/bash
# Evidence run (round 5): GPU parity suite, smoke, the driver's bench command, rocprof kernel
# stats + PMC passes (scripts/gpu_pmc.sh), the config-4 strong-scaling shard sizes, the other
# BASELINE configs and §8f rows, the end-to-end line from host memory, a two-rank run sharing
# GPU 0 (the multi-rank path with the real engine), the EQ accounting, config-5 and 2048-shard
# kernel traces, the host-sanitized driver's GPU tests and the per-call bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
step bench
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-160
step pmc
bash scripts/gpu_pmc.sh || exit 1
for n in 2048 4096 8192; do
  step n$n
  timeout -k 10 300 python bench.py --npkts $n --steps 40 --warmup 5 --no-cpu > gpurun_out/bench_n$n.log 2>&1 || { tail -5 gpurun_out/bench_n$n.log; exit 1; }
  tail -1 gpurun_out/bench_n$n.log | cut -c1-120
done
for a in "--config 1 --warmup 15" "--config 2 --steps 20 --warmup 15" "--config 5 --steps 20 --warmup 15" "--config 5 --steps 40 --warmup 15" "--eq" "--tx --warmup 15" "--e2e"; do
  step "$a"
  f=gpurun_out/bench_$(echo $a | tr -d ' -').log
  timeout -k 10 300 python bench.py --steps 10 $a > $f 2>&1 || { echo "bench $a failed"; tail -5 $f; exit 1; }
  tail -1 $f | cut -c1-140
done
step share2
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_share2.log 2>&1 || { tail -5 gpurun_out/bench_share2.log; exit 1; }
step eq-accounting
timeout -k 10 300 python scripts/eq_accounting.py > gpurun_out/eq_accounting.json 2>&1 || { tail -5 gpurun_out/eq_accounting.json; exit 1; }
cat gpurun_out/eq_accounting.json
R=$(pwd)
step rocprof-c5-2048
( cd /tmp && export TMPDIR=/tmp && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5 -o run -- python3 $R/bench.py --config 5 --pipeline 1 --steps 10 --warmup 2 --no-cpu > $R/gpurun_out/prof_c5.log 2>&1 && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_n2048 -o run -- python3 $R/bench.py --npkts 2048 --pipeline 1 --steps 20 --warmup 2 --no-cpu > $R/gpurun_out/prof_n2048.log 2>&1 ) || { echo "rocprof failed"; exit 1; }
step asan-driver
ZRX_DRIVER=ziria_amd/_lib/asan/ziria_rx_driver ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  timeout -k 10 300 python -u -m pytest tests/test_driver.py -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/asan_driver.log 2>&1 || { tail -5 gpurun_out/asan_driver.log; exit 1; }
tail -1 gpurun_out/asan_driver.log
step percall
timeout -k 10 120 ziria_amd/_lib/percall_bench 10 1500 > gpurun_out/percall.json 2>&1 || exit 1
echo evidence-ok
