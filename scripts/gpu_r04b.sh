#!/bin/bash
# Round 4: segment tests + the pipeline probe at the config-4 shard sizes (new uniform cut).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_segments.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_seg.log 2>&1 || { tail -30 gpurun_out/pytest_seg.log; exit 1; }
tail -2 gpurun_out/pytest_seg.log
for n in 2048 4096 8192 16384; do
  timeout -k 10 300 python -u scripts/exp/pipeline_probe3.py $n 20 3 > gpurun_out/probe3_$n.log 2>&1 || { tail -20 gpurun_out/probe3_$n.log; exit 1; }
  echo "== $n"; grep -v amdgpu.ids gpurun_out/probe3_$n.log | tail -6
done
echo r04b-ok
