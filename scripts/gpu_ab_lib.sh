#!/bin/bash
# A/B timing of engine builds: runs the default bench once per entry of VARIANTS (names of
# _lib/libziria_rx.NAME.so, "cur" = the in-tree build), interleaved ROUNDS times, and prints
# the data-Viterbi stage time, the chain ms/step and the CRC-pass count of each run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for v in ${VARIANTS:-cur}; do
    if [ "$v" = cur ]; then unset ZRX_LIB_VARIANT; else export ZRX_LIB_VARIANT=$v; fi
    timeout -k 10 200 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab_${v}_$r.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/ab_${v}_$r.log; exit $rc; }
    python -c "
import json
for l in open('gpurun_out/ab_${v}_$r.log'):
    if l.startswith('{'): d=json.loads(l); print('$v', d.get('stage_ms', {}).get('data_viterbi'), d['ms_per_step'], d['value'], d.get('bit_exact_check', d.get('frames_equal_sent')))"
  done
done
