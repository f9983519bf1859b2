#!/bin/bash
# A/B of k_data_fft waves per block (ZRX_DF_WAVES 2 / 1 with one LUT copy: 4 / 8 blocks per CU)
# against the in-tree library on config 5 and config 3; variants built with build_flags_variant.sh.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for A in "--config 5" ""; do for r in 1 2 3; do
  for v in cur w2 w1; do
    if [ "$v" = cur ]; then unset ZRX_LIB_VARIANT; else export ZRX_LIB_VARIANT=$v; fi
    timeout -k 10 200 python bench.py $A --steps 40 --warmup 10 --no-cpu --no-sub > gpurun_out/seg.log 2>&1 || { tail -3 gpurun_out/seg.log; exit 1; }
    python -c "
import json
l=[x for x in open('gpurun_out/seg.log') if x.startswith('{')]
d=json.loads(l[-1])
print('$v', d['stage_ms']['data_fft_demap'], d['ms_per_step'], d['value'], d.get('value_one_engine'), d['bit_exact_check']['payload_match'], d['bit_exact_check']['crc_pass'])"
  done
done; done
