#!/bin/bash
# A/B of ZRX_SEG_MIX_NUM (mixed-batch segment length, zrx_viterbi3.hpp) on config 5: build the
# variants first with scripts/build_flags_variant.sh mN "-DZRX_SEG_MIX_NUM=N" (N = 9, 10, 12, 13).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for r in 1 2 3; do
  for v in cur m9 m10 m12 m13; do
    if [ "$v" = cur ]; then unset ZRX_LIB_VARIANT; else export ZRX_LIB_VARIANT=$v; fi
    timeout -k 10 200 python bench.py --config 5 --steps 40 --warmup 10 --no-cpu --no-sub > gpurun_out/seg.log 2>&1 || { tail -3 gpurun_out/seg.log; exit 1; }
    python -c "
import json
l=[x for x in open('gpurun_out/seg.log') if x.startswith('{')]
d=json.loads(l[-1])
print('$v', d['stage_ms']['data_viterbi'], d['ms_per_step'], d['value'], d.get('value_one_engine'), d['bit_exact_check']['payload_match'], d['bit_exact_check']['crc_pass'])"
  done
done
