#!/bin/bash
# Round 4: LDS tables staged with every load in flight at once (k_data_fft, k_descramble_crc,
# k_signal_fft) against the previous commit (prev); then the stall PMC passes on the current
# sources for every chain kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
VARIANTS="cur prev" ROUNDS=3 STEPS=20 AB_TAG=m3 bash scripts/gpu_ab_lib.sh || exit 1
bash scripts/gpu_pmc_stall.sh || exit 1
python scripts/pmc_stall_summary.py gpurun_out/stall_summary.json
