#!/bin/bash
# Config 5, packed plan, one engine: what a frame's final traceback costs (experiment builds,
# wrong output): exp = product kernel (DBG 0) and no final tracebacks (DBG 4096).  (Round 6 also
# timed their argmin without the walks, -DZRX_NO_FINAL_WALK: about half of the cost; PERFLOG.)
# Data-Viterbi stage of engine 0, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in exp:0 exp:4096; do
    lib=${v%%:*}; d=${v##*:}
    ZRX_LIB_VARIANT=$lib ZRX_V3DBG=$d timeout -k 10 200 python bench.py --config 5 --pipeline 1 --steps 10 --warmup 5 \
      --no-cpu --no-sub > gpurun_out/fin_${lib}_${d}_$r.log 2>&1 || { tail -3 gpurun_out/fin_${lib}_${d}_$r.log; exit 1; }
    python -c "
import json
l=[x for x in open('gpurun_out/fin_${lib}_${d}_$r.log') if x.startswith('{')]
d=json.loads(l[-1])
print('$lib dbg $d', d['stage_ms']['data_viterbi'], d['ms_per_step'])"
  done
done
