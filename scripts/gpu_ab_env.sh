#!/bin/bash
# A/B timing of one environment knob: runs the default bench once per value of $VALUES for
# the variable $VAR, interleaved ROUNDS times; prints the Viterbi stage time, the chain
# ms/step, the value and the bit-exact check of each run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for v in ${VALUES}; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu ${BENCH_ARGS:-} > gpurun_out/abenv_${v}_$r.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/abenv_${v}_$r.log; exit $rc; }
    python -c "
import json
for l in open('gpurun_out/abenv_${v}_$r.log'):
    if l.startswith('{'): d=json.loads(l); sm=d.get('stage_ms', {}); print('$VAR=$v', sm.get('data_viterbi'), sm.get('descramble_crc'), d['ms_per_step'], d['value'], (d.get('bit_exact_check') or {}).get('payload_match'))"
  done
done
