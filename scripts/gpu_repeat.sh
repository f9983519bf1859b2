#!/bin/bash
# Config 5 evidence line again (value_one_engine now unlinked).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config 5 --steps 10 > gpurun_out/bench_config5.log 2>&1 || { tail -5 gpurun_out/bench_config5.log; exit 1; }
tail -1 gpurun_out/bench_config5.log | cut -c1-200
python -c "
import json
for l in open('gpurun_out/bench_config5.log'):
    if l.startswith('{'): d=json.loads(l); print(d['value'], d['value_one_engine'], d['ms_per_step'], d['pipeline'])"
