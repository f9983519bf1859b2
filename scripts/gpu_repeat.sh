#!/bin/bash
# HIP stream priority range on this box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 120 python -c "
import torch
print('torch priority_range', torch.cuda.Stream.priority_range())
import ctypes
h = ctypes.CDLL('libamdhip64.so')
lo, hi = ctypes.c_int(), ctypes.c_int()
print('hip', h.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi)), lo.value, hi.value)
"
