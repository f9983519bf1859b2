#!/bin/bash
# Younger-wave issue priority around 2/3 (cur): 3/5, 5/8, 5/7, 7/10; config 3, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
VARIANTS="cur p35 p58 p57 p710" ROUNDS=3 STEPS=20 AB_TAG=u3 bash scripts/gpu_ab_lib.sh || exit 1
