#!/bin/bash
# Builds the engine of git revision REV as ziria_amd/_lib/libziria_rx.NAME.so for A/B timing
# on the GPU box (ZRX_LIB_VARIANT=NAME python bench.py ...; see scripts/gpu_ab_lib.sh).
# usage: scripts/build_variant.sh REV NAME ["-DFLAGS ..."]
set -euo pipefail
REV=$1; NAME=$2; FLAGS=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
git -C "$ROOT" archive "$REV" ziria_amd/csrc include | tar -x -C "$TMP"
python3 "$TMP/ziria_amd/csrc/gen_tables.py"
OBJS=""
for f in zrx_host zrx_ext_cxx; do
  if [ -f "$TMP/ziria_amd/csrc/$f.cpp" ]; then
    g++ -O3 -std=c++17 -fPIC -c "$TMP/ziria_amd/csrc/$f.cpp" -o "$TMP/$f.o"
    OBJS="$OBJS $TMP/$f.o"
  fi
done
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -pthread -DZRX_EXPERIMENTS $FLAGS -o "$ROOT/ziria_amd/_lib/libziria_rx.$NAME.so" \
  "$TMP/ziria_amd/csrc/zrx_api.hip" ${OBJS:+-x none $OBJS}
echo "$ROOT/ziria_amd/_lib/libziria_rx.$NAME.so"
