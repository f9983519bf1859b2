"""Probe: config-3 steps with 1 or 2 engines (streams) over 1 or 2 distinct input batches,
each setting measured 3x interleaved (host wall time around 40 steps), plus per-step GPU
times from HIP events on the engines' streams."""
import sys
import time

import torch

sys.path.insert(0, ".")
from ziria_amd import txgen  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402

bs = [txgen.make_batch_range(0, 16384, seed=0x5EED + j, sigma=4.0, device="cuda") for j in range(2)]
S = max(b["max_nsym"] for b in bs)
engs = [RxEngine(0), RxEngine(0)]
strs = [torch.cuda.Stream(), torch.cuda.Stream()]
outs = []
for e in engs:
    e.reserve(16384, S)
    outs.append((torch.zeros((16384, 4096), dtype=torch.uint8, device="cuda"),
                 torch.zeros((16384, 8), dtype=torch.int32, device="cuda")))
for st in strs:
    st.wait_stream(torch.cuda.current_stream())


def run(k, ne, nb, ev=None):
    for i in range(k):
        j, bi = i % ne, i % nb
        with torch.cuda.stream(strs[j]):
            if ev is not None:
                ev[i][0].record()
            engs[j].rx(bs[bi]["sym"], bs[bi]["sym_off"], bs[bi]["nsym"], S, outs[j][0], outs[j][1])
            if ev is not None:
                ev[i][1].record()


for rep in range(3):
    for ne, nb in ((1, 1), (1, 2), (2, 1), (2, 2)):
        run(4, ne, nb)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(40, ne, nb)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        run(10, ne, nb, ev)
        torch.cuda.synchronize()
        gpu = sorted(a.elapsed_time(b) for a, b in ev)
        print(f"engines {ne} batches {nb}: {dt / 40 * 1e3:.4f} ms/step wall, {16384 * 1500 * 8 * 40 / dt / 1e9:.1f} "
              f"Gbit/s; per-step span median {gpu[5]:.3f} ms", flush=True)
