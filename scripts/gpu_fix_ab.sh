#!/bin/bash
# A/B of the working tree's engine (curx: experiment build of the tree) against another
# revision's (old: scripts/build_variant.sh REV old): the shards of config 4 (2048 and 4096
# packets), config 3, config 5 and config 2, interleaved;
# data-Viterbi stage, ms/step, Gbit/s.  (Round 6: tree = the packed-plan sources, old = 180f4e3;
# PERFLOG §F "Packed plan".)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in curx old; do
    export ZRX_LIB_VARIANT=$v
    for a in "--npkts 2048" "--npkts 4096" "" "--config 5" "--config 2"; do
      extra=""
      true
      timeout -k 10 200 python bench.py $a $extra --steps 60 --payload 1500 --warmup 15 --batches 2 --no-cpu --no-sub > gpurun_out/fx.log 2>&1 || { tail -3 gpurun_out/fx.log; exit 1; }
      python -c "
import json
l=[x for x in open('gpurun_out/fx.log') if x.startswith('{')]
d=json.loads(l[-1])
print('$v', '$a', d.get('stage_ms', {}).get('data_viterbi'), d['ms_per_step'], d['value'])"
    done
  done
done
