#!/bin/bash
# Timing experiment: k_viterbi3 with parts switched off (ZRX_V3DBG bits; outputs wrong for
# nonzero values, timing only).  Prints the data-Viterbi stage time of each variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for d in ${DBGS:-0 1 2 4 8 16}; do
  ZRX_V3DBG=$d timeout -k 10 200 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu > gpurun_out/dbg_$d.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "dbg $d rc=$rc"; tail -5 gpurun_out/dbg_$d.log; exit $rc; }
  python -c "
import json
for l in open('gpurun_out/dbg_$d.log'):
    if l.startswith('{'): d=json.loads(l); print('dbg=$d', d['stage_ms']['data_viterbi'], d['bit_exact_check']['crc_pass'])"
done
