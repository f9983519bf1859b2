#!/bin/bash
# A/B of an experiment build (ZRX_LIB_VARIANT=$1, scripts/build_flags_variant.sh) against the
# in-tree library (cur): the variant's GPU parity tests first, then 3 interleaved rounds of
# config 5, config 3, --eq and the 2048-packet shard; the data-FFT stage and ms/step.
V=$1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ZRX_LIB_VARIANT=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_eq.py tests/test_gpu_fullsize.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/${V}_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/${V}_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in cur $V; do
    if [ "$v" = cur ]; then unset ZRX_LIB_VARIANT; else export ZRX_LIB_VARIANT=$v; fi
    for a in "--config 5" "" "--eq" "--npkts 2048 --steps 60"; do
      timeout -k 10 200 python bench.py --steps 30 $a --warmup 10 --no-cpu --no-sub > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 1; }
      python -c "
import json
l=[x for x in open('gpurun_out/ab.log') if x.startswith('{')]
d=json.loads(l[-1])
print('$v', '$a', d.get('stage_ms', {}).get('data_fft_demap'), d['ms_per_step'], d['value'], d['bit_exact_check'].get('payload_match', d['bit_exact_check']))"
    done
  done
done
