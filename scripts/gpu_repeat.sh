#!/bin/bash
# Link mode 8 (the chain's tail on a high-priority stream) and 12 (8 + the head on a low one)
# against mode 4 and one engine, config 5, interleaved; linked-engine parity first.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "linked" --timeout 120 --timeout-method thread > gpurun_out/pytest_link.log 2>&1 || { tail -20 gpurun_out/pytest_link.log; exit 1; }
tail -1 gpurun_out/pytest_link.log
for r in 1 2; do
  for a in "--pipeline 1" "--pipeline 2 --link 4" "--pipeline 2 --link 8" "--pipeline 2 --link 12" "--pipeline 2 --link 9"; do
    f=gpurun_out/rep_c5_$(echo $a | tr -d ' -')_$r.log
    timeout -k 10 200 python bench.py --config 5 --no-cpu --warmup 3 --steps 30 $a > $f 2>&1 || exit 1
    python -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('c5 $a', d['value'], d['ms_per_step'], d.get('value_one_engine'))"
  done
done
