"""Probe: K config-3 steps on one engine vs alternating between two engines on two streams."""
import time, torch, sys
sys.path.insert(0, ".")
from ziria_amd import txgen
from ziria_amd.engine import RxEngine
b = txgen.make_batch(16384, seed=0x5EED, sigma=4.0, device="cuda")
engs = [RxEngine(0), RxEngine(0)]
strs = [torch.cuda.Stream(), torch.cuda.Stream()]
outs = []
for e in engs:
    e.reserve(16384, b["max_nsym"])
    outs.append((torch.zeros((16384, 4096), dtype=torch.uint8, device="cuda"),
                 torch.zeros((16384, 8), dtype=torch.int32, device="cuda")))
def run(k, n):
    for i in range(k):
        j = i % n
        with torch.cuda.stream(strs[j]):
            engs[j].rx(b["sym"], b["sym_off"], b["nsym"], b["max_nsym"], outs[j][0], outs[j][1])
for n in (1, 2, 1, 2, 1, 2):
    run(4, n); torch.cuda.synchronize()
    t0 = time.perf_counter(); run(40, n); torch.cuda.synchronize(); dt = time.perf_counter() - t0
    print(n, "engines: %.4f ms/step, %.1f Gbit/s" % (dt / 40 * 1e3, 16384 * 1500 * 8 * 40 / dt / 1e9), flush=True)
print("same outputs:", bool((outs[0][0] == outs[1][0]).all()), bool((outs[0][1] == outs[1][1]).all()))
