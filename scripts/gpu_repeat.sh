#!/bin/bash
# Config 5 evidence line, 40 steps (10-step lines carry the first steps' transient).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config 5 --steps 40 > gpurun_out/bench_config5.log 2>&1 || { tail -5 gpurun_out/bench_config5.log; exit 1; }
python -c "
import json
for l in open('gpurun_out/bench_config5.log'):
    if l.startswith('{'): d=json.loads(l); print(d['value'], d['value_one_engine'], d['ms_per_step'], d['pipeline'], d['bit_exact_check'] if 'bit_exact_check' in d else '', d.get('cpu_baseline'))" | cut -c1-400
