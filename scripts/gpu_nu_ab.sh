#!/bin/bash
# k_data_fft with its store loop sized by the widest soft row of the wave (nu: the working
# tree's build) against the committed kernel (cur): GPU parity of the variant first, then
# interleaved config 5, config 3 and the 2048-packet shard; the data-FFT stage and ms/step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ZRX_LIB_VARIANT=nu timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_eq.py tests/test_gpu_fullsize.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/nu_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/nu_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in cur nu; do
    if [ "$v" = cur ]; then unset ZRX_LIB_VARIANT; else export ZRX_LIB_VARIANT=$v; fi
    for a in "--config 5" "" "--npkts 2048 --steps 60"; do
      timeout -k 10 200 python bench.py --steps 30 $a --warmup 10 --no-cpu --no-sub > gpurun_out/nu.log 2>&1 || { tail -3 gpurun_out/nu.log; exit 1; }
      python -c "
import json
l=[x for x in open('gpurun_out/nu.log') if x.startswith('{')]
d=json.loads(l[-1])
print('$v', '$a', d.get('stage_ms', {}).get('data_fft_demap'), d['ms_per_step'], d['value'], d['bit_exact_check'].get('payload_match', d['bit_exact_check']))"
    done
  done
done
