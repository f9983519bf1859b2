"""Probe: config-3 steps with one engine, or two engines on their own streams taking the
steps in turn with each zrx_pipeline_link mode (0 none, 1 Viterbi after the peer's chain,
2 data FFT after the peer's Viterbi, 3 both), interleaved, `reps` rounds of each; host wall
time around `steps` steps between synchronizes (the bench's timed region).
python scripts/exp/pipeline_probe3.py [npkts] [steps] [reps]"""
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
engs = [RxEngine(0), RxEngine(0)]
strs = [torch.cuda.Stream(), torch.cuda.Stream()]
outs = []
for e in engs:
    e.reserve(n, S)
    outs.append((torch.zeros((n, 4096), dtype=torch.uint8, device="cuda"),
                 torch.zeros((n, 8), dtype=torch.int32, device="cuda")))
for st in strs:
    st.wait_stream(torch.cuda.current_stream())
bits = n * 1500 * 8


def run(k, ne):
    for i in range(k):
        j, bi = i % ne, i % 2
        with torch.cuda.stream(strs[j]):
            engs[j].rx(bs[bi]["sym"], bs[bi]["sym_off"], bs[bi]["nsym"], S, outs[j][0], outs[j][1])


modes = [(1, 0), (2, 0), (2, 1), (2, 2), (2, 3)]
res = {m: [] for m in modes}
for rep in range(reps):
    for ne, lm in modes:
        engs[0].link(engs[1], lm) if lm else engs[0].link(engs[1], 0)
        run(4, ne)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(steps, ne)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[(ne, lm)].append(dt / steps * 1e3)
        print(f"rep {rep} engines {ne} link {lm}: {dt / steps * 1e3:.4f} ms/step, {bits * steps / dt / 1e9:.1f} Gbit/s",
              flush=True)
engs[0].link(engs[1], 0)
for m, v in res.items():
    v = sorted(v)
    print(f"engines {m[0]} link {m[1]}: ms/step min {v[0]:.4f} median {v[len(v) // 2]:.4f} max {v[-1]:.4f}; "
          f"Gbit/s at median {bits / v[len(v) // 2] / 1e6:.1f}", flush=True)
for j in range(2):                     # batch 0 on both engines
    with torch.cuda.stream(strs[j]):
        engs[j].rx(bs[0]["sym"], bs[0]["sym_off"], bs[0]["nsym"], S, outs[j][0], outs[j][1])
torch.cuda.synchronize()
print("engines' outputs equal:", bool((outs[0][0] == outs[1][0]).all()) and bool((outs[0][1] == outs[1][1]).all()))
