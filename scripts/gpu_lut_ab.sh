#!/bin/bash
# k_data_fft with the demap LUT read once per lane before the modulation switch (cur) against
# reading it inside each modulation's branch (lut0: -DZRX_DF_LUT_ONCE=0), interleaved: config
# 5 (mixed modulations in a wave), config 3 and --eq; the data-FFT stage and ms/step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in cur lut0; do
    if [ "$v" = cur ]; then unset ZRX_LIB_VARIANT; else export ZRX_LIB_VARIANT=$v; fi
    for a in "--config 5" "" "--eq"; do
      timeout -k 10 200 python bench.py $a --steps 30 --warmup 10 --no-cpu --no-sub > gpurun_out/lut.log 2>&1 || { tail -3 gpurun_out/lut.log; exit 1; }
      python -c "
import json
l=[x for x in open('gpurun_out/lut.log') if x.startswith('{')]
d=json.loads(l[-1])
print('$v', '$a', d.get('stage_ms', {}).get('data_fft_demap'), d['ms_per_step'], d['value'])"
    done
  done
done
