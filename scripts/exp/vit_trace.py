"""Probe (ZRX_VTRACE build: scripts/build_flags_variant.sh vtrace -DZRX_VTRACE): the k_viterbi3
timeline of one config-5 batch and one config-3 batch.  Every row records its wave's start
and end (s_memrealtime, 100 MHz), HW_ID / XCC_ID, block, columns and rate; saved to
gpurun_out/vtrace_<cfg>.npz with a per-SIMD summary printed: when each SIMD went idle,
how many waves it ran, how the rows' columns spread over the SIMDs."""
import ctypes
import os
import sys

os.environ["ZRX_LIB_VARIANT"] = "vtrace"
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, ".")
from ziria_amd import txgen  # noqa: E402
from ziria_amd._lib import lib  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402

dev = torch.device("cuda", 0)
eng = RxEngine(0)
vtrace_set = lib().zrx_vtrace_set
vtrace_set.argtypes = [ctypes.c_void_p, ctypes.c_int]   # (a 64-bit device pointer, not a C int)
vtrace_set.restype = ctypes.c_int
os.makedirs("gpurun_out", exist_ok=True)


def trace(name, b):
    n = b["nsym"].numel()
    S = b["max_nsym"]
    eng.reserve(n, S)
    pay = torch.zeros((n, 4096), dtype=torch.uint8, device=dev)
    info = torch.zeros((n, 8), dtype=torch.int32, device=dev)
    for _ in range(3):
        eng.rx(b["sym"], b["sym_off"], b["nsym"], S, pay, info)
    torch.cuda.synchronize()
    buf = torch.zeros(65536 * 8, dtype=torch.int32, device=dev)
    assert vtrace_set(buf.data_ptr(), 65536) == 0
    eng.rx(b["sym"], b["sym_off"], b["nsym"], S, pay, info)
    torch.cuda.synchronize()
    assert vtrace_set(None, 0) == 0
    rows, fixes = eng.plan_stats()
    t = buf.view(-1, 8)[:rows].cpu().numpy().astype(np.int64)
    np.savez_compressed(f"gpurun_out/vtrace_{name}.npz", t=t, rows=rows, fixes=fixes)
    t = t[t[:, 0] != 0]                                  # (slots a chained plan left empty)
    rows = t.shape[0]
    t0 = t[:, 0] - t[:, 0].min()
    t1 = t[:, 1] - t[:, 0].min()
    hw, xcc = t[:, 2], t[:, 3]
    simd = (xcc & 15) * 1024 + ((hw >> 13) & 7) * 128 + ((hw >> 12) & 1) * 64 + ((hw >> 8) & 15) * 4 + ((hw >> 4) & 3)
    span = t1.max()
    ends = {}
    waves = {}
    cols = {}
    for i in range(rows):
        s = int(simd[i])
        ends[s] = max(ends.get(s, 0), int(t1[i]))
        waves.setdefault(s, set()).add((int(t[i, 4]), int(t0[i])))
        cols[s] = cols.get(s, 0) + int(t[i, 5])
    e = np.array(sorted(ends.values()))
    c = np.array(list(cols.values()))
    nw = np.array([len(v) for v in waves.values()])
    print(f"{name}: rows {rows} fixes {fixes} simds {len(ends)} span {span / 100:.1f} us; "
          f"SIMD idle at (us) p0 {e[0] / 100:.1f} p10 {np.percentile(e, 10) / 100:.1f} "
          f"p50 {np.percentile(e, 50) / 100:.1f} p90 {np.percentile(e, 90) / 100:.1f} max {e[-1] / 100:.1f}; "
          f"waves per SIMD min {nw.min()} max {nw.max()}; columns per SIMD min {c.min()} mean {c.mean():.0f} "
          f"max {c.max()}; wave starts after 5 us: {int((t0 > 500).sum())} rows", flush=True)
    busy = np.zeros(int(span) // 10 + 1)
    for i in range(0, rows, 8):
        busy[int(t0[i]) // 10:int(t1[i]) // 10 + 1] += 1
    print("  waves running per 10 us (of 2048 slots):", " ".join(str(int(x)) for x in busy[::5][:400]), flush=True)


trace("c5", txgen.make_mixed_fast(16384, min_len=64, max_len=4095, sigma=3.0, seed=0x3C5, device=dev))
trace("c3", txgen.make_batch_range(0, 16384, seed=0x5EED, sigma=4.0, device=dev))
