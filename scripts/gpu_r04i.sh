#!/bin/bash
# Round 4: config 5 two-engine regression hunt: SIGNAL FFT block shape (cur 16 lanes, sig64)
# and the engines' link mode, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in cur sig64 prev; do
    for lk in 0 1; do
      if [ "$v" = cur ]; then unset ZRX_LIB_VARIANT; else export ZRX_LIB_VARIANT=$v; fi
      timeout -k 10 200 python bench.py --config 5 --steps 10 --warmup 2 --cpu-seconds 0.2 --link $lk > gpurun_out/c5_${v}_${lk}_$r.log 2>&1 || { tail -5 gpurun_out/c5_${v}_${lk}_$r.log; exit 1; }
      python -c "
import json
for l in open('gpurun_out/c5_${v}_${lk}_$r.log'):
    if l.startswith('{'): d=json.loads(l); print('$v link $lk', d['ms_per_step'], d['value'], d['stage_ms'])"
    done
  done
done
echo r04i-ok
