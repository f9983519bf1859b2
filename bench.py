"""Benchmark: decoded payload Mbit/s of the 802.11a 54 Mbps RX hot path on MI355X.

One step = one pass of the whole HIP chain (SIGNAL FFT+demap, SIGNAL Viterbi + header,
data FFT + demap + deinterleave, data Viterbi, descramble + CRC) over one batch of
synthetic time-domain packets already resident in HBM (BASELINE config 3: 16384 packets x
1500 B payload at 54 Mbps = 57 OFDM symbols each).  Multi-GPU: one process per GPU, each
rank decodes its own 16384-packet batch (weak scaling, no collective in the hot loop);
after the timed region the CRC-pass counts are all-reduced and the payload bytes gathered
to rank 0 over RCCL (ziria_amd/node.py).

Stage times come from HIP events recorded by the engine on its own stream around every
kernel of every timed step (zrx_enable_timing), so `roofline.achieved` is measured live
over the timed region.  `roofline.traffic` is the per-launch HBM byte count from the
rocprofv3 PMC passes summarised in profiles/pmc_summary.json (scripts/pmc_summary.py).

python bench.py [--gpus N --steps K --warmup W]   (N>1 under torch.distributed.run)
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from ziria_amd import node, txgen  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402

VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12   # 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz = 78.6
HBM_PEAK_GBS = 8000.0
OPS_PER_DECODED_BIT = 256                       # 64 ACS x (add, add, compare, select)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_summary.json")


def traffic_for(kernel, npkts):
    """HBM bytes per launch of `kernel` from the committed PMC summary (same workload)."""
    try:
        s = json.load(open(PMC_SUMMARY))
        k = s["kernels"][kernel]
        if int(s.get("npkts", -1)) != npkts:
            return None
        return k.get("hbm_bytes_per_launch")
    except (OSError, KeyError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--npkts", type=int, default=16384)
    ap.add_argument("--payload", type=int, default=1500)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="wall time budget of the CPU baseline")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if world > 1:
            dist.barrier()

    # ---------------------------------------------------------------- workload (HBM-resident)
    b = txgen.make_batch(args.npkts, mod=3, coding=2, payload_len=args.payload,
                         seed=0x5EED + 7919 * rank, device=dev)
    n, S = args.npkts, b["max_nsym"]
    eng = RxEngine(local)
    eng.reserve(n, S)
    payload = torch.zeros((n, 4096), dtype=torch.uint8, device=dev)
    info = torch.zeros((n, 8), dtype=torch.int32, device=dev)

    def step():
        eng.rx(b["sym"], b["sym_off"], b["nsym"], S, payload, info)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    eng.enable_timing(True)                       # stage events on the engine's stream, every step
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    stage = eng.stage_ms()                        # averages over the K timed steps
    eng.enable_timing(False)
    elapsed = node.max_over_ranks(t1 - t0, device=dev)

    # ---------------------------------------------------------------- bit-exact self-check + gather
    ok, bits, match = node.counts(info, payload=payload, expected=b["payload"])
    torch.cuda.synchronize()
    tg = time.perf_counter()
    ok_all, bits_all, match_all, _ = node.combine(ok, bits, match, payload[:, :args.payload].contiguous(),
                                                  device=dev)
    torch.cuda.synchronize()
    gather_ms = (time.perf_counter() - tg) * 1e3 if world > 1 else 0.0

    decoded_bits = n * (args.payload + 4 + 2) * 8          # Viterbi output bits per launch
    vit_ms = stage["data_viterbi"]
    achieved_tops = OPS_PER_DECODED_BIT * decoded_bits / (vit_ms * 1e-3) / 1e12
    nsym_data = S - 1
    fft_bytes = n * nsym_data * (256 + 288)                # complex16 symbol in + 64-QAM soft out
    fft_gbs = fft_bytes / (stage["data_fft_demap"] * 1e-3) / 1e9

    value = bits_all * args.steps / elapsed / 1e6          # CRC-checked payload bits, all ranks
    ms_per_step = elapsed / args.steps * 1e3

    # ---------------------------------------------------------------- CPU baseline (rank 0, N=1)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(b, args.payload, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "decoded Mbit/s (whole node) 802.11a 54Mbps RX, bit-exact, at 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "Mbit/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int16+u8",
            "data": "synthetic (txgen: random payloads, TX restated from transmitter.blk, AWGN sigma=4)",
            "config": {"workload": f"config3: {n} packets/GPU x {args.payload} B payload @ 54 Mbps "
                                   f"(64-QAM r3/4), {S} CP-removed complex16 OFDM symbols each, "
                                   "time-domain input resident in HBM",
                       "packets_per_gpu": n, "payload_bytes": args.payload, "symbols_per_packet": S,
                       "parallelism": f"packet-sharded x{world}"},
            "bit_exact_check": {"crc_pass": ok_all, "packets": n * world, "payload_match": match_all == world},
            "stage_ms": {k: round(v, 4) for k, v in stage.items()},
            "roofline": {"kernel": "k_viterbi3 (data Viterbi)", "bound": "valu",
                         "achieved": round(achieved_tops, 3), "peak": round(VALU_PEAK_TOPS, 1),
                         "unit": "Tops/s", "frac": round(achieved_tops / VALU_PEAK_TOPS, 4),
                         "traffic": traffic_for("k_viterbi3", n),
                         "units": f"{OPS_PER_DECODED_BIT} int ops per decoded bit x {decoded_bits} bits/launch"},
            "roofline_fft": {"kernel": "k_data_fft (FFT64+GetData+demap+deinterleave)", "bound": "hbm",
                             "achieved": round(fft_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(fft_gbs / HBM_PEAK_GBS, 4),
                             "traffic": traffic_for("k_data_fft", n),
                             "units": f"544 B per data symbol x {n * nsym_data} symbols/launch"},
            "gather_ms": round(gather_ms, 3),
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(b, payload_len, seconds):
    """The oracle (scalar C restatement, "port") on the host cores this process may use,
    packet-parallel with pthreads, over chunks of the same packets until `seconds` of wall
    time have passed."""
    from oracle import oracle as O
    threads = min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count() or 1)
    sym = b["sym"].cpu().numpy()
    off_all = b["sym_off"].cpu().numpy()
    ns_all = b["nsym"].cpu().numpy()
    chunk = 1024
    done = ok = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        lo = done % off_all.size
        hi = min(lo + chunk, off_all.size)
        _, res = O.rx_batch_time(sym, off_all[lo:hi], ns_all[lo:hi], nthreads=threads)
        ok += sum(r["crc_ok"] for r in res)
        done += hi - lo
    dt = time.perf_counter() - t0
    bits = ok * payload_len * 8
    return {"value": round(bits / dt / 1e6, 2), "unit": "Mbit/s", "cores": threads, "kind": "port",
            "sample": f"{done} packets of the same batch ({ok} CRC-ok), {dt:.1f} s wall on {threads} threads"}


if __name__ == "__main__":
    main()
