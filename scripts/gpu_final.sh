#!/bin/bash
# Round-6 evidence session on the final sources: the GPU parity suite and smoke(), the default
# bench line (headline + sub-results), --e2e, --eq, --tx, --config 1, then the rocprof kernel
# trace and PMC passes of the headline (scripts/gpu_pmc.sh -> gpurun_out/pmc_summary.json), and
# the kernel trace of config 5 on one engine.
# Outputs go to gpurun_out/final_*; copy what is judged into profiles/r06/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
run() {   # name, limit, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/final_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; tail -1 gpurun_out/final_$n.log | cut -c1-300
  return $rc
}
if [ -z "$SKIP_PYTEST" ]; then
  step pytest
  run pytest_gpu 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread || exit 1
  step smoke
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
step bench
run bench_default 400 python -u bench.py --steps 20 --warmup 15 || exit 1
[ -n "$ONLY_BENCH" ] && exit 0
step e2e
run bench_e2e 300 python -u bench.py --e2e --steps 10 --warmup 3 || exit 1
step eq
run bench_eq 300 python -u bench.py --eq --steps 20 --warmup 15 || exit 1
step tx
run bench_tx 300 python -u bench.py --tx --steps 20 --warmup 15 --cpu-seconds 5 || exit 1
step config1
run bench_config1 300 python -u bench.py --config 1 --steps 20 --warmup 15 --cpu-seconds 5 || exit 1
if [ -z "$SKIP_PMC" ]; then
  step pmc
  ./scripts/gpu_pmc.sh > gpurun_out/final_pmc.log 2>&1; rc=$?
  echo "pmc rc=$rc"; tail -3 gpurun_out/final_pmc.log; [ $rc -eq 0 ] || exit $rc
  python scripts/kstats.py gpurun_out/prof/run_kernel_stats.csv
fi
if [ -z "$SKIP_C5PROF" ]; then
  step c5prof
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/c5prof" -o c5 -- python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" \
     --config 5 --pipeline 1 --steps 20 --warmup 5 --no-cpu --no-sub > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/final_c5prof.log" 2>&1); rc=$?
  echo "c5prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python scripts/kstats.py gpurun_out/c5prof/c5_kernel_stats.csv
fi
exit 0
