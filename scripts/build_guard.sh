#!/bin/bash
# Debug build of the working tree with ZRX_GUARD (range-checked Viterbi stores, printed
# instead of faulting): ziria_amd/_lib/libziria_rx.guard.so, loaded with ZRX_LIB_VARIANT=guard.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DZRX_GUARD -o "$ROOT/ziria_amd/_lib/libziria_rx.guard.so" \
  "$ROOT/ziria_amd/csrc/zrx_api.hip"
