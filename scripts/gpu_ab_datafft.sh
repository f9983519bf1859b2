cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in st w4; do
  ZRX_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_$v.log 2>&1 || { echo "$v tests failed"; tail -20 gpurun_out/pt_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/pt_$v.log)"
done
for r in 1 2; do
  for v in cur st w4; do
    if [ "$v" = cur ]; then unset ZRX_LIB_VARIANT; else export ZRX_LIB_VARIANT=$v; fi
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/ab_${v}_$r.log 2>&1 || { echo "$v bench failed"; tail -5 gpurun_out/ab_${v}_$r.log; exit 1; }
    python -c "
import json
for l in open('gpurun_out/ab_${v}_$r.log'):
    if l.startswith('{'): d=json.loads(l); print('$v', d['stage_ms']['data_fft_demap'], d['ms_per_step'], d['value'], d['bit_exact_check']['payload_match'])"
  done
done
