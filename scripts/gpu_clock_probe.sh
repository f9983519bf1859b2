#!/bin/bash
# Per-dispatch effective clock of the chain's kernels over a long run (GRBM_GUI_ACTIVE / 8 /
# duration, MI355X_MICROARCH.md DVFS notes): does k_viterbi3 speed up over consecutive
# launches because the clock rises, or for another reason?
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/clk -o clk -- python3 $R/bench.py --steps 40 --warmup 2 --no-cpu --pipeline 1 > $R/gpurun_out/clk.log 2>&1; echo rc=$?
