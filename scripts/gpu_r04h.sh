#!/bin/bash
# Round 4: tail kernels (SIGNAL FFT block shape, CRC lane-shift tables, plan reuse) -- GPU
# parity suite, rocprof kernel stats of the working tree, A/B against HEAD (prev).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_h -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu > $R/gpurun_out/prof_h.log 2>&1 || { tail -5 $R/gpurun_out/prof_h.log; exit 1; }
cd $R
grep -E "k_signal|k_pkt|k_descr|k_data|k_viterbi3" gpurun_out/prof_h/run_kernel_stats.csv | cut -d, -f1-4
VARIANTS="cur prev" ROUNDS=3 STEPS=20 AB_TAG=c3 bash scripts/gpu_ab_lib.sh || exit 1
VARIANTS="cur prev" ROUNDS=2 STEPS=10 AB_TAG=c5 BENCH_ARGS="--config 5 --cpu-seconds 0.5" bash scripts/gpu_ab_lib.sh || exit 1
ZRX_LIB_VARIANT=snap timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_segments.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_snap.log 2>&1 || { tail -20 gpurun_out/pytest_snap.log; exit 1; }
tail -1 gpurun_out/pytest_snap.log
echo r04h-ok
