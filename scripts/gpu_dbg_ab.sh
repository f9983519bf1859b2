cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for r in 1 2 3; do
for d in 0 1 2048; do
  ZRX_LIB_VARIANT=exp ZRX_V3DBG=$d timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/dbg_${d}_$r.log 2>&1; rc=$?
  python -c "
import json
l=[x for x in open('gpurun_out/dbg_${d}_$r.log') if x.startswith('{')]
d=json.loads(l[-1]) if l else {}
print('dbg $d', d.get('stage_ms',{}).get('data_viterbi'), d.get('ms_per_step'), d.get('bit_exact_check',{}).get('payload_match'))" || tail -3 gpurun_out/dbg_${d}_$r.log
done
done
