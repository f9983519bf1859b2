#!/bin/bash
# Builds the working tree's engine with extra compile flags as ziria_amd/_lib/libziria_rx.NAME.so
# for A/B timing on the GPU box (ZRX_LIB_VARIANT=NAME; scripts/gpu_ab_lib.sh).
# usage: scripts/build_flags_variant.sh NAME "-DFOO=1 -DBAR=2"
set -euo pipefail
NAME=$1; FLAGS=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
cd "$ROOT/ziria_amd/csrc"
for f in zrx_host zrx_ext_cxx; do g++ -O3 -std=c++17 -fPIC -c $f.cpp -o "$TMP/$f.o"; done
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $FLAGS -o "$ROOT/ziria_amd/_lib/libziria_rx.$NAME.so" \
  zrx_api.hip -x none "$TMP/zrx_host.o" "$TMP/zrx_ext_cxx.o"
echo "$ROOT/ziria_amd/_lib/libziria_rx.$NAME.so"
