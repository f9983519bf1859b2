#!/bin/bash
# Round 4: ZRX_V3DBG attribution of the guard-free Viterbi (experiment build of HEAD).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
LIBV=exp DBGS="0 1 2 4 8 16 1024 0" bash scripts/gpu_dbg_sweep.sh || exit 1
echo r04d-ok
