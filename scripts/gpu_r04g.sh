#!/bin/bash
# Round 4: HIP-graph replay vs eager launches of the chain, and the pipeline probe after the
# faster Viterbi.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/exp/graph_probe.py 16384 20 4 > gpurun_out/graph_probe.log 2>&1 || { tail -20 gpurun_out/graph_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/graph_probe.log | tail -4
timeout -k 10 300 python -u scripts/exp/graph_probe.py 2048 40 3 > gpurun_out/graph_probe_2k.log 2>&1 || { tail -20 gpurun_out/graph_probe_2k.log; exit 1; }
grep -v amdgpu.ids gpurun_out/graph_probe_2k.log | tail -4
timeout -k 10 300 python -u scripts/exp/pipeline_probe3.py 16384 20 3 > gpurun_out/probe3_16384b.log 2>&1 || { tail -20 gpurun_out/probe3_16384b.log; exit 1; }
grep -v amdgpu.ids gpurun_out/probe3_16384b.log | tail -6
echo r04g-ok
