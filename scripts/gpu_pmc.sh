#!/bin/bash
# tests + bench + PMC passes given in $PMC1, $PMC2 (space-separated counter lists)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; ok $rc || exit $rc
python - <<'PY'
import json
for l in open("gpurun_out/bench.log"):
    if l.startswith("{"):
        d = json.loads(l); print(d["value"], d["ms_per_step"], d["stage_ms"], d["roofline"]["frac"], d["bit_exact_check"])
PY
cd /tmp && export TMPDIR=/tmp
[ -f $R/gpurun_out/counters.txt ] || timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1
i=0
for P in "$PMC1" "$PMC2" "$PMC3"; do
  [ -z "$P" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmc$i -o pmc -- python3 $R/bench.py --npkts ${PMC_NPKTS:-4096} --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/pmc$i.log 2>&1; rc=$?
  echo "pmc$i rc=$rc"; ok $rc || exit $rc
done
exit 0
