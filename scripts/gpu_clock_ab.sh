cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
 for c in 1 0; do
  for cfg in "--config 2" "--config 5" "--npkts 4096 --no-sub"; do
   ZRX_BENCH_STEPCLOCK=$c timeout -k 10 200 python bench.py $cfg --steps 20 --warmup 15 --no-cpu --cpu-seconds 0.1 > gpurun_out/clk_${c}_$r.log 2>&1 || exit 1
   python -c "
import json,sys
for l in open('gpurun_out/clk_${c}_$r.log'):
    if l.startswith('{'): d=json.loads(l); print('clock=$c', '$cfg', d['value'], d['ms_per_step'], d.get('value_one_engine'))"
  done
 done
done
