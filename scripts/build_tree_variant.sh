#!/bin/bash
# Builds the working tree's engine with one text substitution applied (A/B of an uncommitted
# change): scripts/build_tree_variant.sh NAME FILE OLD_TEXT_FILE NEW_TEXT_FILE
# (OLD_TEXT_FILE "-": NEW_TEXT_FILE replaces the whole of FILE)
# -> ziria_amd/_lib/libziria_rx.NAME.so (ZRX_EXPERIMENTS build, as build_variant.sh).
set -euo pipefail
NAME=$1; FILE=$2; OLD=$3; NEW=$4
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
mkdir -p "$TMP/ziria_amd" "$TMP/include"
cp -r "$ROOT/ziria_amd/csrc" "$TMP/ziria_amd/"
cp "$ROOT/include/ziria_rx.h" "$TMP/include/"
python3 - "$TMP/ziria_amd/csrc/$FILE" "$OLD" "$NEW" <<'PY'
import sys
p, o, n = sys.argv[1:]
s = open(p).read(); new = open(n).read()
if o == "-":
    s = new
else:
    old = open(o).read()
    assert old in s, "old text not found"
    s = s.replace(old, new)
open(p, "w").write(s)
PY
cd "$TMP/ziria_amd/csrc"
python3 gen_tables.py
for f in zrx_host zrx_ext_cxx; do g++ -O3 -std=c++17 -fPIC -c $f.cpp -o "$TMP/$f.o"; done
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -pthread -DZRX_EXPERIMENTS -o "$ROOT/ziria_amd/_lib/libziria_rx.$NAME.so" \
  zrx_api.hip -x none "$TMP/zrx_host.o" "$TMP/zrx_ext_cxx.o"
echo "$ROOT/ziria_amd/_lib/libziria_rx.$NAME.so"
