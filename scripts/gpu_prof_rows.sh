#!/bin/bash
# rocprofv3 kernel-trace stats of the §8f workloads: config 3 + eq (ChannelEqualization +
# PilotTrack fused into the FFT kernels) and config 1 (the RX front end over captures).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_eq -o run -- python3 $R/bench.py --eq --steps 10 --warmup 2 --no-cpu > $R/gpurun_out/prof_eq.log 2>&1; rc=$?
echo "eq rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c1 -o run -- python3 $R/bench.py --config 1 --steps 10 --warmup 2 > $R/gpurun_out/prof_c1.log 2>&1; rc=$?
echo "c1 rc=$rc"
