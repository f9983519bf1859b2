#!/bin/bash
# A/B of k_data_fft variants (scripts/build_flags_variant.sh builds): chain parity per
# variant, then interleaved bench rounds (scripts/gpu_ab_lib.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  [ "$v" = cur ] && continue
  ZRX_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_eq.py -m gpu -x -q --timeout 120 --timeout-method thread -k "chain or eq" > gpurun_out/pt_$v.log 2>&1 || { echo "$v tests failed"; tail -20 gpurun_out/pt_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/pt_$v.log)"
done
ROUNDS=${ROUNDS:-2} STEPS=${STEPS:-10} bash scripts/gpu_ab_lib.sh
