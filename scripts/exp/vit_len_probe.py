"""Probe: k_viterbi3 throughput (trellis columns per second) on uniform batches of short to
long frames at rates 1/2 and 3/4, ~200 M columns a batch, soft = 7*coded + U[-2,2].
Tells whether short rows cost more per column than config 3's 1500-byte ones."""
import sys

import torch

sys.path.insert(0, ".")
from ziria_amd import txgen  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402

dev = torch.device("cuda", 0)
eng = RxEngine(0)
for cr in (0, 2):
    for fl in (64, 128, 256, 512, 1024, 1500, 2048):
        nbits = 8 * fl + 6
        L = -(-nbits // 72) * 72
        n = int(150e6 // L)
        gen = torch.Generator(device=dev)
        gen.manual_seed(fl)
        u = torch.zeros((n, L), dtype=torch.uint8, device=dev)
        u[:, :8 * fl] = torch.randint(0, 2, (n, 8 * fl), generator=gen, device=dev, dtype=torch.uint8)
        coded = txgen._encode(u, cr).to(torch.int16)
        del u
        noise = torch.randint(-2, 3, coded.shape, generator=gen, device=dev, dtype=torch.int16)
        soft = torch.clamp(coded * 7 + noise, 0, 7).to(torch.int8).contiguous()
        del coded, noise
        ns = soft.shape[1]
        soft = soft.reshape(-1)
        cols = ns // (2 if cr == 0 else 4) * (cr + 1)
        soft_off = torch.arange(n, dtype=torch.int64, device=dev) * ns
        params = torch.tensor([fl, cr, ns, 0], dtype=torch.int32, device=dev).repeat(n, 1).contiguous()
        stride = -(-fl // 16) * 16
        out = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
        out_off = torch.arange(n, dtype=torch.int64, device=dev) * stride
        out_bits = torch.zeros(n, dtype=torch.int32, device=dev)
        eng.reserve(n, 1)
        for _ in range(3):
            eng.viterbi(soft, soft_off, params, out, out_off, out_bits)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for _ in range(10):
            eng.viterbi(soft, soft_off, params, out, out_off, out_bits)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 10
        ok = bool((out_bits == 8 * fl).all())
        print(f"rate {cr} fl {fl:5d} frames {n:7d} cols {cols:6d}: {ms:.4f} ms, "
              f"{n * cols / ms / 1e6:.1f} G col/s, ok {ok}", flush=True)
        del soft, out
