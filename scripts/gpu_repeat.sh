#!/bin/bash
# Config 2 (Viterbi only): one engine against two in flight, interleaved; config 5 default.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for a in "--config 2 --pipeline 1" "--config 2 --pipeline 2"; do
    f=gpurun_out/rep_$(echo $a | tr -d ' -')_$r.log
    timeout -k 10 200 python bench.py --no-cpu --warmup 3 --steps 30 $a > $f 2>&1 || exit 1
    python -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$a', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 200 python bench.py --config 5 --steps 20 --cpu-seconds 0.5 > gpurun_out/rep_c5_default.log 2>&1 || exit 1
python -c "
import json
for l in open('gpurun_out/rep_c5_default.log'):
    if l.startswith('{'): d=json.loads(l); print('c5 default', d['value'], d['ms_per_step'], d['pipeline'], d.get('oracle_sample_match'))"
