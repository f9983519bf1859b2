#!/bin/bash
# Round 4, first session: pipeline-link A/B (one process, interleaved), a kernel trace of the
# pipelined default bench, and the strong-scaling shard sizes of config 4 on one GPU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/exp/pipeline_probe3.py 16384 20 4 > gpurun_out/probe3_16k.log 2>&1 || { tail -20 gpurun_out/probe3_16k.log; exit 1; }
tail -6 gpurun_out/probe3_16k.log
for n in 2048 4096 8192; do
  timeout -k 10 300 python bench.py --npkts $n --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_n$n.log 2>&1 || { tail -20 gpurun_out/bench_n$n.log; exit 1; }
  tail -1 gpurun_out/bench_n$n.log | cut -c1-200
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $R/gpurun_out/trace_bench.log 2>&1 || { tail -5 $R/gpurun_out/trace_bench.log; exit 1; }
echo r04a-ok
