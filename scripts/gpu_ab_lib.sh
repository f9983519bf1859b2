#!/bin/bash
# A/B timing of engine builds: runs the default bench once per entry of VARIANTS (names of
# _lib/libziria_rx.NAME.so, "cur" = the in-tree build), interleaved ROUNDS times, and prints
# the data-Viterbi stage time, the chain ms/step and the CRC-pass count of each run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for v in ${VARIANTS:-cur}; do
    if [ "$v" = cur ]; then unset ZRX_LIB_VARIANT; else export ZRX_LIB_VARIANT=$v; fi
    timeout -k 10 200 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu --no-sub ${BENCH_ARGS:-} > gpurun_out/ab${AB_TAG:-}_${v}_$r.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/ab${AB_TAG:-}_${v}_$r.log; exit $rc; }
    python -c "
import json
for l in open('gpurun_out/ab${AB_TAG:-}_${v}_$r.log'):
    if l.startswith('{'): d=json.loads(l); sm=d.get('stage_ms', {}); print('$v', sm.get('data_viterbi'), sm.get('data_fft_demap'), sm.get('signal_viterbi'), sm.get('descramble_crc'), d['ms_per_step'], d['value'], d.get('bit_exact_check', {}).get('payload_match') if 'bit_exact_check' in d else d.get('frames_equal_sent'))"
  done
done
