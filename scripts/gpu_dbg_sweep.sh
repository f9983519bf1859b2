#!/bin/bash
# Times the default bench under each ZRX_V3DBG timing-experiment variant in $DBGS to
# attribute the Viterbi kernel's overheads (1 no traceback walk, 2 no snapshot stores,
# 4 no normalize, 8 no P broadcast, 16 no event checks, 1024 no soft fetch); the output of
# those variants is wrong by design.  LIBV = library variant, BENCH_ARGS = bench workload.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for d in ${DBGS:-0 1 2 8 16 0}; do
  ZRX_LIB_VARIANT=${LIBV:-} ZRX_V3DBG=$d timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu ${BENCH_ARGS:-} > gpurun_out/dbg_$d.log 2>&1 || exit 1
  python - "$d" <<'PY'
import json, sys
for l in open(f"gpurun_out/dbg_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l); print("dbg", sys.argv[1], d.get("stage_ms", {}).get("data_viterbi"), d["ms_per_step"], d.get("bit_exact_check"))
PY
done
