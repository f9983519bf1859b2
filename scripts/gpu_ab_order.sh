#!/bin/bash
# A/B: bench with and without the k_vit_order packet ordering, alternating, on one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for o in 1 0 1 0; do
  ZRX_ORDER=$o timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/ab_$o.log 2>&1 || exit 1
  python -c "
import json
d = json.loads([l for l in open('gpurun_out/ab_$o.log') if l.startswith('{')][-1])
print('order=$o', d['stage_ms']['data_viterbi'], d['value'])"
done
