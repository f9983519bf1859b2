#!/bin/bash
# Config 5 with the packed plan (ZRX_FILL=1) and rows of frames (ZRX_FILL=0), each with the
# product Viterbi and without its tracebacks (experiment build, ZRX_V3DBG=1: wrong output, a
# timing probe): the data-Viterbi stage time of engine 0 alone, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  for f in 1 0; do
    for d in ${DBGS:-0 1}; do
      ZRX_FILL=$f ZRX_LIB_VARIANT=exp ZRX_V3DBG=$d timeout -k 10 200 python bench.py --config 5 --pipeline 1 --steps 10 --warmup 5 \
        --no-cpu --no-sub > gpurun_out/fab_${f}_${d}_$r.log 2>&1 || { tail -3 gpurun_out/fab_${f}_${d}_$r.log; exit 1; }
      python -c "
import json
l=[x for x in open('gpurun_out/fab_${f}_${d}_$r.log') if x.startswith('{')]
d=json.loads(l[-1])
print('fill $f dbg $d', d['stage_ms']['data_viterbi'], d['ms_per_step'], d['bit_exact_check']['payload_match'])"
    done
  done
done
