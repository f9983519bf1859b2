#!/bin/bash
# Link mode 4 (the chain's head on a low-priority stream): config 5 and a 4096-packet config-3
# shard, interleaved against one engine and the other link modes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "linked or plan" --timeout 120 --timeout-method thread > gpurun_out/pytest_link.log 2>&1 || { tail -20 gpurun_out/pytest_link.log; exit 1; }
tail -1 gpurun_out/pytest_link.log
run() {
  f=gpurun_out/rep_$(echo "$*" | tr -d ' -')_$r.log
  timeout -k 10 200 python bench.py --no-cpu --warmup 3 --steps 30 "$@" > $f 2>&1 || exit 1
  python -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$*', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
  for a in "--pipeline 1" "--pipeline 2 --link 0" "--pipeline 2 --link 4" "--pipeline 2 --link 6" "--pipeline 2 --link 5"; do
    run --config 5 $a
  done
done
for r in 1 2; do
  for a in "--pipeline 1" "--pipeline 2 --link 1" "--pipeline 2 --link 5" "--pipeline 2 --link 4"; do
    run --npkts 4096 $a
  done
done
