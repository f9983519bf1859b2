cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
LIBV=exp DBGS="0 1 2 4 8 1024 0" BENCH_ARGS="--pipeline 1" bash scripts/gpu_dbg_sweep.sh || exit 1
timeout -k 10 300 python scripts/exp/vit_trace.py > gpurun_out/vtrace.log 2>&1; rc=$?; cat gpurun_out/vtrace.log | cut -c1-1500; exit $rc
