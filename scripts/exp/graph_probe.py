"""Probe: config-3 steps launched eagerly (six kernels per step through zrx_rx_dev) against the
same chain captured once into a HIP graph (torch.cuda.CUDAGraph around engine.rx) and
replayed, interleaved; host wall time around `steps` steps between synchronizes.
python scripts/exp/graph_probe.py [npkts] [steps] [reps]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from ziria_amd import txgen  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
bs = [txgen.make_batch_range(0, n, seed=0x5EED + j, sigma=4.0, device="cuda") for j in range(2)]
S = max(b["max_nsym"] for b in bs)
eng = RxEngine(0)
eng.reserve(n, S)
pay = torch.zeros((n, 4096), dtype=torch.uint8, device="cuda")
info = torch.zeros((n, 8), dtype=torch.int32, device="cuda")
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
bits = n * 1500 * 8


def eager(k):
    with torch.cuda.stream(s):
        for i in range(k):
            b = bs[i % 2]
            eng.rx(b["sym"], b["sym_off"], b["nsym"], S, pay, info)


eager(4)
torch.cuda.synchronize()
graphs = []
for j in range(2):                       # one graph per input batch
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        b = bs[j]
        eng.rx(b["sym"], b["sym_off"], b["nsym"], S, pay, info)
    graphs.append(g)
torch.cuda.synchronize()


def graphed(k):
    with torch.cuda.stream(s):
        for i in range(k):
            graphs[i % 2].replay()


res = {"eager": [], "graph": []}
for rep in range(reps):
    for name, fn in (("eager", eager), ("graph", graphed)):
        fn(3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[name].append(dt / steps * 1e3)
        print(f"rep {rep} {name}: {dt / steps * 1e3:.4f} ms/step, {bits * steps / dt / 1e9:.1f} Gbit/s", flush=True)
for k, v in res.items():
    v = sorted(v)
    print(f"{k}: ms/step min {v[0]:.4f} median {v[len(v) // 2]:.4f}; Gbit/s at median {bits / v[len(v) // 2] / 1e6:.1f}")
graphs[0].replay()
torch.cuda.synchronize()
ref = (pay.clone(), info.clone())
eager(1)
torch.cuda.synchronize()
print("graph output equals eager:", bool((pay == ref[0]).all()) and bool((info == ref[1]).all()))
