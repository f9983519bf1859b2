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

python bench.py [--gpus N --steps K --warmup W]   (N>1: one process per GPU; started under
torch.distributed.run by the caller, or by bench.py itself when WORLD_SIZE is not set)

Secondary workloads (our own reporting, not the driver's line): --config 2 = BASELINE
config 2, the batched Viterbi alone (4096 x 1500-byte frames, rate 1/2, soft input in HBM);
--config 5 = BASELINE config 5, mixed MCS (8 rates, PSDU length 64..4095 B; lengths above
2048 are header errors under the reference parser and carry no payload).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from ziria_amd import node, txgen  # noqa: E402
from ziria_amd._lib import lib as zlib  # noqa: E402
from ziria_amd.build import source_hash  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402

VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12   # 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz = 78.6
HBM_PEAK_GBS = 8000.0
OPS_PER_DECODED_BIT = 256                       # 64 ACS x (add, add, compare, select)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_summary.json")
# Two rx batches in flight pay only while one batch's Viterbi leaves the GPU idle around it:
# interleaved on one box (profiles/r04_pipeline_probe.txt, Gbit/s, one engine / two linked):
# 2048 packets 101.5 / 114.6, 4096 125.2 / 133.3, 8192 140.7 / 131.6, 16384 155.3 / 155.1.
PIPELINE_BELOW = 8192


def pmc_kernel(kernel, npkts):
    """The committed PMC summary's entry for `kernel` when it was measured on the same
    workload and the same kernel sources (csrc_sha256, ziria_amd.build.source_hash); None
    otherwise."""
    try:
        s = json.load(open(PMC_SUMMARY))
        if int(s.get("npkts", -1)) != npkts or s.get("csrc_sha256") != source_hash():
            return None
        return s["kernels"][kernel]
    except (OSError, KeyError, ValueError, TypeError):
        return None


def traffic_for(kernel, npkts):
    """HBM bytes per launch of `kernel` from the committed PMC summary (pmc_kernel)."""
    k = pmc_kernel(kernel, npkts)
    return k.get("hbm_bytes_per_launch") if k else None


def rocprof_frac(kernel, npkts, work, peak):
    """The roofline fraction priced on the rocprofv3 kernel trace of the same sources (the
    summary's mean launch duration, clock-ramp launches included, and its median), beside the
    bench's own HIP-event figure: work / duration / peak."""
    k = pmc_kernel(kernel, npkts)
    if not k or not k.get("avg_duration_ns"):
        return None
    out = {"avg_duration_ms": round(k["avg_duration_ns"] / 1e6, 4),
           "frac_avg": round(work / (k["avg_duration_ns"] * 1e-9) / peak, 4),
           "source": "profiles/pmc_summary.json (rocprofv3 --kernel-trace of the same sources)"}
    if k.get("median_duration_ns"):
        out["median_duration_ms"] = round(k["median_duration_ns"] / 1e6, 4)
        out["frac_median"] = round(work / (k["median_duration_ns"] * 1e-9) / peak, 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--npkts", type=int, default=16384, help="packets per GPU (config 3: 16384)")
    ap.add_argument("--total", type=int, default=0,
                    help="global packet count split over the ranks (default npkts x N, i.e. weak scaling)")
    ap.add_argument("--payload", type=int, default=1500)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="wall time budget of the CPU baseline")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pipeline", type=int, default=0, choices=[0, 1, 2],
                    help="batches in flight: 2 = two engines (own workspace and stream) take the steps in "
                         "turn, as a streaming receiver would, so one batch's tail overlaps the next one's head; "
                         "0 (default) = auto: 2 for an rx batch under %d packets per GPU (zrx_pipeline_link "
                         "mode 1) and for configs 2 and 5, else 1" % PIPELINE_BELOW)
    ap.add_argument("--link", type=int, default=-1, choices=list(range(-1, 16)),
                    help="zrx_pipeline_link mode of two engines (-1: auto = 9 for configs 3/4, 4 for config 5)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="with --gpus N: every rank on GPU 0 over a gloo process group (the multi-rank path on a "
                         "one-GPU box; functional, not a scaling point)")
    ap.add_argument("--batches", type=int, default=2,
                    help="distinct input batches per GPU the steps rotate through (config 3/4/5)")
    ap.add_argument("--config", type=int, default=3, choices=[1, 2, 3, 5])
    ap.add_argument("--tx", action="store_true",
                    help="TX chain (transmitter() at 40 MHz, SURVEY §8f row 4) on config-3 packets")
    ap.add_argument("--eq", action="store_true",
                    help="config 3 through a channel, with ChannelEqualization + PilotTrack (SURVEY §8f row 1)")
    ap.add_argument("--no-sub", action="store_true",
                    help="skip the secondary workloads (configs 2 and 5, the 2048/4096-packet shards) the default "
                         "one-GPU line carries as sub_results")
    ap.add_argument("--e2e", action="store_true",
                    help="config 3 end to end from host memory through __ext_wifi_rx_batch (SURVEY §8d: kernel-only "
                         "vs end-to-end incl. H2D from pinned memory)")
    args = ap.parse_args()
    if args.tx:
        return bench_tx(args)
    if args.e2e:
        return bench_e2e(args)
    if args.config == 1:
        return bench_capture(args)
    if args.config == 2:
        return bench_viterbi_only(args, cpu=not args.no_cpu)
    if args.config == 5:
        return bench_mixed(args, cpu=not args.no_cpu)

    world = int(os.environ.get("WORLD_SIZE", "0"))
    if args.gpus > 1 and world == 0:
        return spawn_ranks(args.gpus)                  # before anything touches the GPU
    world = max(world, 1)
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    # --share-gpu: every rank on device 0, the process group over gloo (RCCL refuses two ranks
    # on one device) -- the multi-rank path with the real engine on a one-GPU box; the ranks
    # contend for one GPU, so its numbers are no scaling point
    local = 0 if args.share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.share_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    # The headline: config 3 at N = 1; at N > 1 the driver's SCALE command (no --total) is weak
    # scaling, 16384 packets per rank.  The same N-rank run then also decodes config 4 as SURVEY
    # §8(d) defines it -- config 3's 16384 packets split over the N ranks (strong scaling) --
    # and reports it as "strong", so one SCALE invocation yields both.
    head = rx_run(args, args.total if args.total else args.npkts * world, world, rank, local, dev)
    strong = None
    if world > 1 and not args.total:
        strong = rx_run(args, args.npkts, world, rank, local, dev)

    cpu = None                                         # (the CPU baseline: rank 0 of an N = 1 run only)
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(head["batch0"], args.cpu_seconds, head["batch0"].get("chan"))
    ranks = rank_devices(dev, head["rank_elapsed_s"], local)
    subs = None
    if world == 1 and not args.no_sub and not args.eq and not args.total and not args.share_gpu:
        head.pop("batch0", None)
        subs = sub_results(args, dev)

    if rank == 0:
        line = {
            "metric": "decoded Mbit/s (whole node) 802.11a 54Mbps RX, bit-exact, at 1/2/4/8 MI355X",
            "value": head["value"],
            "unit": "Mbit/s",
            "n_gpus": 1 if args.share_gpu else world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak" if not args.total else "strong",
            "vs_baseline": None,
            "dtype": "int16+u8",
            "data": ("synthetic (txgen.make_batch_range: random payloads, TX restated from transmitter.blk, "
                     + ("3-tap channel + phase drift, AWGN sigma=2" if args.eq else "AWGN sigma=4")
                     + f"; {args.batches} distinct batches per GPU, the steps rotate through them)"),
            "config": head["config"],
            "value_one_engine": head["value_one_engine"],
            "bit_exact_check": head["bit_exact_check"],
            "stage_ms": head["stage_ms"],
            "stage_ms_from": "engine 0 alone over the rotating batches, HIP events, after the warmup and as many "
                             "launches again untimed (the clock ramp), before the timed steps",
            "roofline": head["roofline"],
            "roofline_fft": head["roofline_fft"],
            "gather_ms": head["gather_ms"],
            "step_stats": head["step_stats"],
            "step_stats_one_engine": head["step_stats_one_engine"],
            "devices": ranks,
            "cpu_baseline": cpu,
        }
        if subs is not None:
            line["sub_results"] = subs
        if world > 1:
            line["ranks"] = world
            line["cpu_baseline_note"] = "timed at N = 1 only: see the one-GPU line"
        if args.share_gpu:
            line["multi_rank_mode"] = (f"functional: {world} ranks share GPU 0, process group over gloo (host "
                                       "copies); the ranks contend for one GPU, so this is no scaling point")
        if strong is not None:
            line["strong"] = {k: strong[k] for k in ("value", "ms_per_step", "value_one_engine", "bit_exact_check",
                                                     "gather_ms", "step_stats", "rank_elapsed_s")}
            line["strong"].update(scaling="strong", config=strong["config"],
                                  what="config 4 as SURVEY §8(d) defines it: config 3's 16384 packets split over "
                                       f"the {world} ranks, timed in the same run after the weak-scaling headline")
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def rx_run(args, total, world, rank, local, dev):
    """One N-rank measurement of the rx chain over a global batch of `total` packets
    (node.run_sharded: every rank decodes its contiguous shard, rank 0 checks every gathered
    packet).  Returns the line's per-run fields (rank 0's are complete)."""
    # ---------------------------------------------------------------- workload (HBM-resident)
    # One global batch (BASELINE config 4): packet i depends only on (seed, i), each rank
    # builds and decodes its contiguous shard, rank 0 checks every gathered packet.  Each rank
    # holds args.batches distinct such batches (seeds 0x5EED + b) and the steps rotate through
    # them, so no step re-reads samples the previous one left in the caches (MI355X's 256 MiB
    # Infinity Cache holds a whole 239 MB batch).
    sigma = 2.0 if args.eq else 4.0
    nb = args.batches
    lo, hi = node.shard_range(total, world, rank)
    npipe = args.pipeline or (2 if hi - lo < PIPELINE_BELOW else 1)
    # npipe engines, each with its own workspace and stream, take the steps in turn; every
    # step is still one whole pass of the chain over one batch.  Two engines are linked
    # (zrx_pipeline_link mode 9): one batch's Viterbi starts only once the other batch's
    # Viterbi and seam pass are done, so only the short kernels around it overlap.
    engs = [RxEngine(local) for _ in range(npipe)]
    streams = [torch.cuda.Stream(dev) for _ in range(npipe)]
    if npipe == 2 and args.link != 0:
        engs[0].link(engs[1], 9 if args.link < 0 else args.link)
    eng = engs[0]
    state = {}

    def make_shard(lo, hi):
        bs = [txgen.make_batch_range(lo, hi, mod=3, coding=2, payload_len=args.payload, sigma=sigma,
                                     seed=0x5EED + j, device=dev, channel=args.eq) for j in range(nb)]
        n, S = hi - lo, max(x["max_nsym"] for x in bs)
        for e in engs:
            e.reserve(max(n, 1), S)
        outs = [(torch.zeros((n, 4096), dtype=torch.uint8, device=dev),
                 torch.zeros((n, 8), dtype=torch.int32, device=dev)) for _ in engs]
        # the engines run on their own (non-blocking) streams: order them after the inputs and
        # the zero-filled outputs made on the current stream
        for st in streams:
            st.wait_stream(torch.cuda.current_stream(dev))
        state.update(batches=bs, outs=outs, S=S, n=n)
        return state

    def run_on(j, bi):
        x = state["batches"][bi]
        with torch.cuda.stream(streams[j]):
            engs[j].rx(x["sym"], x["sym_off"], x["nsym"], state["S"], state["outs"][j][0], state["outs"][j][1],
                       chan=x.get("chan"))
        state["last_stream"] = streams[j]

    def step(sh, k):
        run_on(k % len(engs), k % nb)

    clock = StepClock(args.steps)

    def on_step(i):
        clock.mark(i, None if i < 0 else state["last_stream"])

    # stage times: a separate instrumented pass of engine 0 alone over the rotating batches,
    # after the warmup and before the timed steps (the pipelined steps overlap, so their
    # per-stream event spans would include the other batch; the timers' own event records
    # stay out of the timed region)
    # The shader clock climbs from ~2.2 to 2.4 GHz over the first ~10 ms of load after an idle
    # GPU (profiles/r05/clock_probe.txt): the timers start after as many launches again
    # untimed, so they see the clock the timed steps run at (those follow the whole pass).
    def instrumented(on):
        if not on:
            return
        ninst = max(3 * nb, min(args.steps, 10))
        for i in range(ninst):
            run_on(0, i % nb)
        eng.enable_timing(True)
        for i in range(ninst):
            run_on(0, i % nb)
        torch.cuda.synchronize(dev)
        state["stage"] = eng.stage_ms()
        eng.enable_timing(False)

    # after the timed region: batch b decoded by every engine, engine 0's output returned for
    # the per-packet check, the others compared with it
    state["outs_equal"] = True

    def outputs(sh, bi):
        for j in range(len(engs)):
            run_on(j, bi)
        torch.cuda.synchronize(dev)
        o = state["outs"]
        state["outs_equal"] &= all(bool((x[0] == o[0][0]).all()) and bool((x[1] == o[0][1]).all()) for x in o[1:])
        return o[0]

    res = node.run_sharded(total, make_shard, step, outputs,
                           lambda lo, hi, bi: txgen.payloads_range(lo, hi, args.payload, seed=0x5EED + bi),
                           args.steps, args.warmup, args.payload, device=dev, crc_ok_only=args.eq,
                           on_timed=instrumented, nbatches=nb, on_step=on_step)
    step_stats = clock.stats()
    stage = state["stage"]
    n, S = res["hi"] - res["lo"], state["S"]
    for e in engs:                                         # the Viterbi plans dropped no rows (ZRX_EPLAN)
        e.plan_check()
    elapsed = res["elapsed"]

    # the same K steps with engine 0 alone (one batch in flight): the pipelined value above is
    # not a kernel speed-up, this is what the overlap of two batches adds to
    for k in range(max(1, args.warmup)):
        run_on(0, k % nb)
    torch.cuda.synchronize(dev)
    node.barrier(dev)
    clock1 = StepClock(args.steps)
    t0 = time.perf_counter()
    clock1.mark(-1)
    for k in range(args.steps):
        run_on(0, k % nb)
        clock1.mark(k, streams[0])
    torch.cuda.synchronize(dev)
    node.barrier(dev)
    single = node.max_over_ranks(time.perf_counter() - t0, device=dev)
    step_stats_one = clock1.stats()

    decoded_bits = n * (args.payload + 4 + 2) * 8          # Viterbi output bits per launch (this rank)
    vit_ms = stage["data_viterbi"]
    achieved_tops = OPS_PER_DECODED_BIT * decoded_bits / (vit_ms * 1e-3) / 1e12
    nsym_data = S - 1
    fft_bytes = n * nsym_data * (256 + 288)                # complex16 symbol in + 64-QAM soft out
    fft_gbs = fft_bytes / (stage["data_fft_demap"] * 1e-3) / 1e9

    value = res["bits"] * args.steps / elapsed / 1e6       # CRC-checked payload bits, all ranks
    ms_per_step = elapsed / args.steps * 1e3
    out = {
        "value": round(value, 1),
        "ms_per_step": round(ms_per_step, 4),
        "batch0": state["batches"][0],
        "config": {"workload": f"config{'3+eq' if args.eq else ('4' if world > 1 else '3')}: {total} packets "
                               f"({n} per GPU, contiguous shards) x {args.payload} B payload "
                               f"@ 54 Mbps (64-QAM r3/4), {S} CP-removed complex16 OFDM symbols each, "
                               "time-domain input resident in HBM"
                               + (", FFT >>> ChannelEqualization >>> PilotTrack >>> GetData" if args.eq else ""),
                   "packets_total": total, "packets_per_gpu": n, "payload_bytes": args.payload,
                   "symbols_per_packet": S, "parallelism": f"packet-sharded x{world}",
                   "batches_per_gpu": nb,
                   "pipeline": f"{len(engs)} batch{'es' if len(engs) > 1 else ''} in flight"
                               + (" (engines on separate streams, steps in turn, linked: a Viterbi starts after "
                                  "the other batch's Viterbi)" if len(engs) > 1 else "")},
        "value_one_engine": round(res["bits"] * args.steps / single / 1e6, 1),
        "stage_ms": {k: round(v, 4) for k, v in stage.items()},
        "roofline": {"kernel": "k_viterbi3 (data Viterbi)", "bound": "valu",
                     "achieved": round(achieved_tops, 3), "peak": round(VALU_PEAK_TOPS, 1),
                     "unit": "Tops/s", "frac": round(achieved_tops / VALU_PEAK_TOPS, 4),
                     "traffic": None if args.eq else traffic_for("k_viterbi3", n),
                     "units": f"{OPS_PER_DECODED_BIT} int ops per decoded bit x {decoded_bits} bits/launch",
                     "rocprof": None if args.eq else rocprof_frac("k_viterbi3", n, OPS_PER_DECODED_BIT * decoded_bits,
                                                                  VALU_PEAK_TOPS * 1e12)},
        "roofline_fft": {"kernel": "k_data_fft (FFT64+GetData+demap+deinterleave)", "bound": "hbm",
                         "achieved": round(fft_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(fft_gbs / HBM_PEAK_GBS, 4),
                         "traffic": None if args.eq else traffic_for("k_data_fft", n),
                         "units": f"544 B per data symbol x {n * nsym_data} symbols/launch",
                         "rocprof": None if args.eq else rocprof_frac("k_data_fft", n, fft_bytes, HBM_PEAK_GBS * 1e9)},
        "gather_ms": round(res["gather_s"] * 1e3, 3),
        "step_stats": step_stats,
        "step_stats_one_engine": step_stats_one,
        "rank_elapsed_s": [round(x, 6) for x in res["rank_elapsed"]],
    }
    if rank == 0:
        out["bit_exact_check"] = {"crc_pass": res["ok"], "packets": res["packets"],
                                  "payload_match": res["payload_match"],
                                  "mismatched_packets": res["mismatched_packets"],
                                  "pipeline_outputs_equal": state["outs_equal"],
                                  "checked_on": f"rank 0, every gathered packet of all {nb} batches vs its "
                                                "transmitted payload"}
    for e in engs:
        e.close()
    return out


def rank_devices(dev, rank_elapsed, local):
    """Per rank: its device index and PCI address (all-gathered, so a multi-GPU record shows
    that the ranks ran on distinct GPUs) and its own elapsed time over the timed region."""
    p = torch.cuda.get_device_properties(dev)
    mine = [float(local), float(p.pci_domain_id), float(p.pci_bus_id), float(p.pci_device_id)]
    allr = node.all_gather_floats(mine, device=dev)
    return [{"rank": r, "device": int(v[0]), "pci": "%04x:%02x:%02x.0" % (int(v[1]), int(v[2]), int(v[3])),
             "name": p.name if r == 0 else None, "elapsed_s": rank_elapsed[r] if r < len(rank_elapsed) else None}
            for r, v in enumerate(allr)]


def sub_results(args, dev):
    """The secondary workloads on the same GPU, each with its own timing and bit-exact check,
    for the driver's one-GPU line: BASELINE config 2 (batched Viterbi alone), config 5 (mixed
    MCS), and config 4's shard sizes at 8 and 4 GPUs (2048 / 4096 packets of config 3 on one
    GPU).  Each runs as its own child process (this script again, no exec), as it does
    standalone: in one process the streams of the workloads before it would share the
    process's few hardware queues with its own, and two batches in flight would serialize
    (config 5: 94.7 in-process against 108-109 Gbit/s).  No CPU baselines (the headline
    carries its own)."""
    import subprocess
    out = {}
    t0 = time.perf_counter()
    keep = ("value", "unit", "ms_per_step", "value_one_engine", "bit_exact_check", "stage_ms", "step_stats",
            "pipeline", "config")
    # (at least 100 timed steps for the sub-millisecond workloads: a timed region of a few ms
    # would read a one-off host or clock hiccup as a throughput change; config 5 at least 40)
    steps = str(max(args.steps, 100))
    common = ["--warmup", str(args.warmup), "--batches", str(args.batches), "--no-cpu", "--no-sub"]
    jobs = [("config2", ["--config", "2", "--steps", steps, "--payload", str(args.payload),
                         "--npkts", str(args.npkts)], None),
            ("config5", ["--config", "5", "--steps", str(max(args.steps, 40)), "--npkts", str(args.npkts)], None)]
    for g in (8, 4):                                    # (2048 / 4096 packets at config 3's 16384)
        n = max(1, args.npkts // g)
        jobs.append((f"shard_{n}", ["--npkts", str(n), "--steps", steps, "--payload", str(args.payload)],
                     f"config 4's per-GPU shard at {g} GPUs: {n} config-3 packets"))
    for name, extra, what in jobs:
        cmd = [sys.executable, os.path.abspath(sys.argv[0])] + extra + common
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=400)
        lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
        if p.returncode != 0 or not lines:
            out[name] = {"error": f"exit {p.returncode}", "stderr_tail": p.stderr[-800:]}
            continue
        r = json.loads(lines[-1])
        out[name] = {k: r[k] for k in keep if k in r}
        if "step_stats_one_engine" in r:
            out[name]["step_stats_one_engine"] = r["step_stats_one_engine"]
        if what:
            out[name]["what"] = what
        out[name]["command"] = "bench.py " + " ".join(extra + common)
    out["wall_s"] = round(time.perf_counter() - t0, 1)
    return out


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: runs this script again under
    torch.distributed.run, one process per GPU on this node (rendezvous on 127.0.0.1), as a
    child process (no exec: nothing here has touched the GPU yet, and the child re-parses the
    same arguments).  Returns the launcher's exit code, non-zero if any rank failed."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(sys.argv[0])] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    rc = subprocess.call(cmd, env=env)
    if rc:
        print(f"bench.py: torch.distributed.run with {n} ranks exited with {rc}", file=sys.stderr)
    sys.exit(rc)


class StepClock:
    """Per-step times inside a timed region, so that a stall shows on the line that had it: a
    HIP event recorded after every step on the stream that ran it (events created before the
    region) and the host clock at the same points.  gpu_step_ms are the gaps between
    consecutive step completions on the GPU; host_issue_ms the host time spent issuing each
    step (a host that issues slower than the GPU decodes starves the GPU)."""

    def __init__(self, steps):
        self.off = os.environ.get("ZRX_BENCH_STEPCLOCK", "1") == "0"     # (A/B of the clock's own cost)
        if self.off:
            return
        self.ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        for e in self.ev:                                # (the HIP events exist before the region)
            e.record()
        torch.cuda.synchronize()
        self.host = [0.0] * (steps + 1)

    def mark(self, i, stream=None):
        """i = -1 at the start of the region, else after timed step i (on its stream)."""
        if self.off:
            return
        self.ev[i + 1].record(stream if stream is not None else torch.cuda.current_stream())
        self.host[i + 1] = time.perf_counter()

    def stats(self):
        if self.off:
            return None
        torch.cuda.synchronize()
        done = sorted(self.ev[0].elapsed_time(e) for e in self.ev[1:])
        g = np.diff([0.0] + done)
        h = np.diff(self.host) * 1e3
        q = lambda a, f: round(float(f(a)), 4) if len(a) else None
        return {"gpu_step_ms": {"min": q(g, np.min), "median": q(g, np.median), "max": q(g, np.max),
                                "mean": q(g, np.mean)},
                "host_issue_ms": {"median": q(h, np.median), "max": q(h, np.max)},
                "slowest_step": int(np.argmax(g)) if len(g) else None,
                "gpu_steps_ms": [round(float(x), 4) for x in g],
                "how": "HIP event after each timed step on its stream; gaps between consecutive completions"}


def _timed(step, steps, warmup, clock=None):
    """warmup untimed steps, then `steps` timed ones; step() returns the stream it launched on
    (or None), which the clock records on."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if clock:
        clock.mark(-1)
    for i in range(steps):
        st = step()
        if clock:
            clock.mark(i, st)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def bench_viterbi_only(args, emit=True, cpu=True):
    """BASELINE config 2: 4096 frames of 1500 bytes, rate 1/2, soft = 7*bit + U[-2,2] clipped
    to [0,7], 24048 soft values per frame (48-value groups), all resident in HBM.
    args.batches distinct batches (the steps rotate through them, so no step re-reads the
    previous step's soft values from L2/MALL) and args.pipeline engines on their own streams
    taking the steps in turn, as in main(); every frame of every batch is checked."""
    from oracle import oracle as O
    dev = torch.device("cuda", 0)
    n = args.npkts if args.npkts != 16384 else 4096
    fl = args.payload
    nb = args.batches
    nbits = 8 * fl + 6
    L = -(-nbits // 24) * 24                                  # 24 input bits per 48 soft values
    stride = -(-fl // 16) * 16
    batches = []
    for j in range(nb):
        gen = torch.Generator(device=dev)
        gen.manual_seed(0x5EED + j)
        u = torch.zeros((n, L), dtype=torch.uint8, device=dev)
        u[:, :8 * fl] = torch.randint(0, 2, (n, 8 * fl), generator=gen, device=dev, dtype=torch.uint8)
        coded = txgen._encode(u, 0).to(torch.int16)
        noise = torch.randint(-2, 3, coded.shape, generator=gen, device=dev, dtype=torch.int16)
        soft = torch.clamp(coded * 7 + noise, 0, 7).to(torch.int8).contiguous()
        ns = soft.shape[1]
        batches.append((soft.reshape(-1), torch.from_numpy(np.packbits(u[:, :8 * fl].cpu().numpy(), axis=1,
                                                                       bitorder="little"))))
        del u, coded, noise
    soft_off = torch.arange(n, dtype=torch.int64, device=dev) * ns
    params = torch.tensor([fl, 0, ns, 0], dtype=torch.int32, device=dev).repeat(n, 1).contiguous()
    out_off = torch.arange(n, dtype=torch.int64, device=dev) * stride
    engs = [RxEngine(0) for _ in range(args.pipeline or 2)]
    streams = [torch.cuda.Stream(dev) for _ in engs]
    outs = []
    for e in engs:
        e.reserve(n, 1)
        outs.append((torch.zeros(n * stride, dtype=torch.uint8, device=dev),
                     torch.zeros(n, dtype=torch.int32, device=dev)))
    for st in streams:                                        # inputs come from the current stream
        st.wait_stream(torch.cuda.current_stream(dev))
    k = {"i": 0}

    def run_on(j, bi):
        with torch.cuda.stream(streams[j]):
            engs[j].viterbi(batches[bi][0], soft_off, params, outs[j][0], out_off, outs[j][1])
        return streams[j]

    def step():
        st = run_on(k["i"] % len(engs), k["i"] % nb)
        k["i"] += 1
        return st
    clock = StepClock(args.steps)
    elapsed = _timed(step, args.steps, args.warmup, clock)
    match = True
    for bi in range(nb):                                      # every batch once more on every engine
        for j in range(len(engs)):
            run_on(j, bi)
        torch.cuda.synchronize()
        for o, ob in outs:
            match &= bool((o.reshape(n, stride)[:, :fl].cpu() == batches[bi][1]).all()) and bool((ob == 8 * fl).all())
    soft = batches[0][0]
    bits = n * fl * 8
    line = {
        "metric": "decoded Mbit/s, batched K=7 rate-1/2 Viterbi only (BASELINE config 2)",
        "value": round(bits * args.steps / elapsed / 1e6, 1), "unit": "Mbit/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (random bits, 802.11a encoder, soft 7*bit+U[-2,2])",
        "config": {"workload": f"config2: {n} frames x {fl} B, R=1/2, {ns} soft values each", "batches": nb},
        "bit_exact_check": {"frames_equal_sent": match, "checked": f"every frame of all {nb} batches, every engine"},
        "pipeline": (f"{len(engs)} batches in flight (engines on separate streams, steps in turn)" if len(engs) > 1
                     else "1 batch in flight"),
        "step_stats": clock.stats(),
    }
    for e in engs:
        e.close()
    if not cpu:
        if emit:
            print(json.dumps(line), flush=True)
        return line
    # CPU port (AVX-512 brick loop, identical to the oracle) on every allowed core, chunks of
    # the same frames for about --cpu-seconds
    threads, host = host_cpus()
    s_np = soft.cpu().numpy()
    chunk = min(n, max(256, 16 * threads))
    c_off = np.arange(chunk, dtype=np.int64) * ns
    c_len, c_fl, c_cr = np.full(chunk, ns, np.int32), np.full(chunk, fl, np.int32), np.zeros(chunk, np.int16)
    c_oo = np.arange(chunk, dtype=np.int64) * (fl + 16)
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds or done == 0:
        lo = (done % (n // chunk)) * chunk
        O.viterbi_batch(s_np[lo * ns:(lo + chunk) * ns], c_off, c_len, c_fl, c_cr, c_oo, chunk * (fl + 16),
                        nthreads=threads, fast=True)
        done += chunk
    cpu_dt = time.perf_counter() - t0
    vit = "AVX-512 vpermb" if O.lib().zp_fft64(None, None, 0) else "scalar"
    line["cpu_baseline"] = {"value": round(done * fl * 8 / cpu_dt / 1e6, 2), "unit": "Mbit/s", "cores": threads,
                            "kind": "port", "per_core": round(done * fl * 8 / cpu_dt / 1e6 / threads, 2), "host": host,
                            "sample": f"{done} frames of the same batch, {cpu_dt:.1f} s wall on {threads} threads (CPU "
                                      f"port: {vit} brick loop, identical to the oracle)"}
    if emit:
        print(json.dumps(line), flush=True)
    return line


def bench_mixed(args, emit=True, cpu=True):
    """BASELINE config 5: mixed MCS batches through the whole chain, every packet distinct
    (txgen.make_mixed_fast); args.batches distinct batches, the steps rotate through them.
    Every CRC-passing payload of every batch is checked against what was sent and a sample of
    batch 0 against the oracle."""
    from oracle import oracle as O
    dev = torch.device("cuda", 0)
    n = args.npkts                                       # 16384, as config 3
    nb = args.batches
    tg = time.perf_counter()
    ms = [txgen.make_mixed_fast(n, min_len=64, max_len=4095, sigma=3.0, seed=0x3C5 + j, device=dev)
          for j in range(nb)]
    gen_s = time.perf_counter() - tg
    S = max(m["max_nsym"] for m in ms)
    # args.pipeline engines (own workspace and stream; auto: 2) take the steps in turn, as in main(),
    # linked in mode 4 by default: each batch's head (SIGNAL, plan, data FFT) on a lowest-priority
    # stream, so the other batch's Viterbi blocks (two block rounds on a mixed batch) are dispatched
    # first.  Interleaved on one box (profiles/r04q_config5_pipeline.txt): one engine 94.6-95.0
    # Gbit/s, two unlinked 75.6-90.3 (the head's blocks took CU room from the Viterbi's second
    # round), two in mode 4 101.3-101.6.
    engs = [RxEngine(0) for _ in range(args.pipeline or 2)]
    streams = [torch.cuda.Stream(dev) for _ in engs]
    link = 4 if args.link < 0 else args.link
    if len(engs) == 2 and link > 0:
        engs[0].link(engs[1], link)
    outs = []
    for e in engs:
        e.reserve(n, S)
        outs.append((torch.zeros((n, 4096), dtype=torch.uint8, device=dev),
                     torch.zeros((n, 8), dtype=torch.int32, device=dev)))
    for st in streams:                                   # inputs and outputs come from the current stream
        st.wait_stream(torch.cuda.current_stream(dev))
    eng = engs[0]
    k = {"i": 0}

    def run_on(j, bi):
        m = ms[bi]
        with torch.cuda.stream(streams[j]):
            engs[j].rx(m["sym"], m["sym_off"], m["nsym"], S, outs[j][0], outs[j][1])
        return streams[j]

    def step():
        st = run_on(k["i"] % len(engs), k["i"] % nb)
        k["i"] += 1
        return st

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ninst = max(3 * nb, min(args.steps, 10))             # stage times: engine 0 alone, before the timed steps,
    for i in range(ninst):                               # after as many launches untimed (the clock ramp, as main())
        run_on(0, i % nb)
    eng.enable_timing(True)
    for i in range(ninst):
        run_on(0, i % nb)
    torch.cuda.synchronize()
    stage = eng.stage_ms()
    eng.enable_timing(False)
    first = k["i"]
    clock = StepClock(args.steps)
    elapsed = _timed(step, args.steps, 0, clock)
    timed_batches = [(first + i) % nb for i in range(args.steps)]
    single = None
    if len(engs) > 1:                                    # the same batches with engine 0 alone, for comparison
        if link > 0:
            engs[0].link(engs[1], 0)                     # (alone and unlinked: plain one-engine launches)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for bi in timed_batches:
            run_on(0, bi)
        torch.cuda.synchronize()
        single = time.perf_counter() - t0
    # every batch decoded once more by every engine: per-packet checks, engines compared
    outs_equal, good, crc_pass, expect_ok, bits_b, infos, pays = True, True, 0, 0, [], [], []
    for bi, m in enumerate(ms):
        for j in range(len(engs)):
            run_on(j, bi)
        torch.cuda.synchronize()
        outs_equal &= all(bool((o[0] == outs[0][0]).all()) and bool((o[1] == outs[0][1]).all()) for o in outs[1:])
        inf = outs[0][1].cpu().numpy().copy()          # (a copy: on a CPU test stub .cpu() aliases)
        pay = outs[0][0].cpu().numpy().copy()
        ok = inf[:, 4] == 1
        good &= all((pay[i, :len(m["payload"][i])] == m["payload"][i]).all() for i in range(n) if ok[i])
        crc_pass += int(ok.sum())
        expect_ok += int((m["meta"][:, 2] <= 2048).sum())
        bits_b.append(int(((inf[:, 2] - 4) * 8 * ok).sum()))
        infos.append(inf)
        pays.append(pay)
    bits = sum(bits_b[bi] for bi in timed_batches) / args.steps
    threads, host = host_cpus()
    sample = min(1024, n)
    m0, inf, pay = ms[0], infos[0], pays[0]
    soff, sn = m0["sym_off"][:sample].cpu().numpy(), m0["nsym"][:sample].cpu().numpy()
    sym_s = m0["sym"][:int((soff + sn).max())].cpu().numpy()
    opay, res = O.rx_batch_time(sym_s, soff, sn, nthreads=threads)
    cpu = cpu_baseline(m0, args.cpu_seconds) if cpu else None
    oracle_match = all(int(inf[i, 4]) == r["crc_ok"] and int(inf[i, 2]) == r["len"] and
                       (not r["crc_ok"] or (pay[i, :r["len"] - 4] == opay[i, :r["len"] - 4]).all())
                       for i, r in enumerate(res))
    for e in engs:
        e.close()
    line = {
        "metric": "decoded Mbit/s, mixed-MCS 802.11a RX chain (BASELINE config 5)",
        "value": round(bits * args.steps / elapsed / 1e6, 1), "unit": "Mbit/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int16+u8",
        "data": f"synthetic (txgen.make_mixed_fast: {nb} batches of {n} distinct packets, 8 MCS, PSDU 64..4095 B, "
                f"AWGN sigma=3; generated in {gen_s:.1f} s; the steps rotate through the batches)",
        "config": {"workload": f"config5: {n} packets per batch, {S} symbols max, "
                               f"{int(ms[0]['nsym'].sum())} symbols in batch 0", "batches": nb},
        "bit_exact_check": {"crc_pass": crc_pass, "expected_crc_pass": expect_ok, "payload_match": good,
                            "oracle_sample": sample, "oracle_sample_match": bool(oracle_match),
                            "pipeline_outputs_equal": outs_equal, "checked": f"every packet of all {nb} batches"},
        "pipeline": (f"{len(engs)} batches in flight (engines on separate streams, steps in turn, zrx_pipeline_link "
                     f"mode {link})" if len(engs) > 1 else "1 batch in flight"),
        "value_one_engine": round(bits * args.steps / single / 1e6, 1) if single else None,
        "stage_ms": {k: round(v, 4) for k, v in stage.items()},
        "step_stats": clock.stats(),
        "cpu_baseline": cpu,
    }
    if emit:
        print(json.dumps(line), flush=True)
    return line


PCIE5_X16_GBS = 32e9 * 16 * 128 / 130 / 8 / 1e9      # 63.0 GB/s per direction (PCIe 5.0 x16)


def bench_e2e(args):
    """SURVEY §8(d) "kernel-only vs end-to-end (incl. H2D from pinned memory) times": config 3
    batches handed over in host memory to the drop-in's batched external __ext_wifi_rx_batch
    (the call a wplc program makes: host arrays in, payload + info out, synchronous), which
    cuts the batch into chunks and overlaps H2D, the chain and D2H (zrx_hostio.hpp).  Timed
    three ways on the same batches: the device API with everything resident in HBM (the
    headline's kernel-only path), the external from pinned host arrays (value), and from
    pageable ones (numpy: the library copies through pinned slots with a worker pool).  The
    link itself is measured by plain torch copies of one batch's samples and payload slots."""
    dev = torch.device("cuda", 0)
    n, nb, L = args.npkts, args.batches, args.payload
    bs = [txgen.make_batch_range(0, n, mod=3, coding=2, payload_len=L, sigma=4.0, seed=0x5EED + j, device=dev)
          for j in range(nb)]
    S = bs[0]["max_nsym"]
    csr = (np.arange(n + 1, dtype=np.int64) * S).astype(np.int32)
    pin = [b["sym"].cpu().pin_memory() for b in bs]
    page = [b["sym"].cpu().numpy().copy() for b in bs]
    sym_bytes = pin[0].numel() * 2
    outs = {"pinned": (torch.zeros((n, 4096), dtype=torch.uint8).pin_memory(),
                       torch.zeros((n, 8), dtype=torch.int32).pin_memory()),
            "pageable": (np.zeros((n, 4096), np.uint8), np.zeros((n, 8), np.int32))}
    P = lambda a: C.c_void_p(a.data_ptr() if torch.is_tensor(a) else a.ctypes.data)
    c_csr = P(csr)

    def call(x, pay, info):
        rc = zlib().__ext_wifi_rx_batch(P(x), S * n, c_csr, n + 1, P(pay), n * 4096 * 8, P(info), n * 8)
        if rc < 0:
            raise RuntimeError(f"__ext_wifi_rx_batch failed ({rc})")
        return rc

    def timed_calls(srcs, key):
        pay, info = outs[key]
        for k in range(args.warmup):
            call(srcs[k % nb], pay, info)
        t0 = time.perf_counter()
        for k in range(args.steps):
            call(srcs[k % nb], pay, info)
        dt = time.perf_counter() - t0
        good = True                                      # every batch once more, checked
        for j in range(nb):
            call(srcs[j], pay, info)
            p, i = (pay.numpy(), info.numpy()) if torch.is_tensor(pay) else (pay, info)
            good &= bool((i[:, 4] == 1).all()) and bool((p[:, :L] == bs[j]["payload"]).all())
        return dt, good

    # kernel-only: the device API on the same batches, resident in HBM
    eng = RxEngine(0)
    eng.reserve(n, S)
    d_pay = torch.zeros((n, 4096), dtype=torch.uint8, device=dev)
    d_info = torch.zeros((n, 8), dtype=torch.int32, device=dev)
    it = {"k": 0}

    def dstep():
        b = bs[it["k"] % nb]
        eng.rx(b["sym"], b["sym_off"], b["nsym"], S, d_pay, d_info)
        it["k"] += 1
    k_dt = _timed(dstep, args.steps, args.warmup)
    # the link alone: one batch's samples up, its payload slots (what the external returns) down
    d_sym = torch.empty_like(bs[0]["sym"])
    h_pay = outs["pinned"][0]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for _ in range(2):
        ev[0].record()
        for j in range(4):
            d_sym.copy_(pin[j % nb], non_blocking=True)
        ev[1].record()
        for j in range(4):
            h_pay.copy_(d_pay, non_blocking=True)
        ev[2].record()
        torch.cuda.synchronize()
    h2d_gbs = 4 * sym_bytes / (ev[0].elapsed_time(ev[1]) * 1e-3) / 1e9
    d2h_gbs = 4 * d_pay.numel() / (ev[1].elapsed_time(ev[2]) * 1e-3) / 1e9
    import ziria_amd as Z
    p_dt, p_ok = timed_calls(pin, "pinned")
    Z.set_host_register(0)                              # pageable arrays staged through pinned slots
    g_dt, g_ok = timed_calls(page, "pageable")
    # the same pageable arrays page-locked by the library on first use (mode 2: this process
    # keeps them mapped until it leaves the mode), then copied in place on every later call
    Z.set_host_register(2)
    tr = time.perf_counter()
    for j in range(nb):
        call(page[j], *outs["pageable"])
    reg_first = (time.perf_counter() - tr) / nb
    reg_stats = Z.node_stats()
    r_dt, r_ok = timed_calls(page, "pageable")
    Z.set_host_register(1)                              # (releases them)
    devices = Z.get_devices()
    bits = n * L * 8
    rate = lambda dt: round(bits * args.steps / dt / 1e6, 1)
    bound = bits / (sym_bytes / (h2d_gbs * 1e9)) / 1e6      # payload Mbit/s if the link ran flat out
    threads, host = host_cpus()
    print(json.dumps({
        "metric": "decoded Mbit/s end to end from host memory, 802.11a 54Mbps RX (config 3 via __ext_wifi_rx_batch)",
        "value": rate(p_dt), "unit": "Mbit/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(p_dt / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int16+u8",
        "data": f"synthetic (txgen.make_batch_range, AWGN sigma=4; {nb} batches, the steps rotate through them)",
        "config": {"workload": f"config3: {n} packets x {L} B @ 54 Mbps, {S} symbols each, "
                               f"{sym_bytes / 1e6:.1f} MB of samples per batch in host memory",
                   "call": "__ext_wifi_rx_batch (synchronous: samples in, payload slots + info out)"},
        "devices": {"shards": devices, "how": "every visible gfx950 device (zrx_get_devices); a call is split "
                                              "into contiguous packet ranges, one host thread, context and PCIe "
                                              "link per device"},
        "end_to_end": {"pinned_Mbps": rate(p_dt), "pageable_Mbps": rate(g_dt),
                       "pageable_registered_Mbps": rate(r_dt),
                       "pageable_registered_frac_of_pinned": round(rate(r_dt) / rate(p_dt), 3),
                       "pageable_first_call_registering_ms": round(reg_first * 1e3, 3),
                       "register_stats_after_first_calls": reg_stats,
                       "pinned_ms_per_batch": round(p_dt / args.steps * 1e3, 3),
                       "pageable_ms_per_batch": round(g_dt / args.steps * 1e3, 3),
                       "pageable_registered_ms_per_batch": round(r_dt / args.steps * 1e3, 3),
                       "kernel_only_Mbps": rate(k_dt), "kernel_only_ms_per_batch": round(k_dt / args.steps * 1e3, 3)},
        "link": {"h2d_GBps": round(h2d_gbs, 1), "d2h_GBps": round(d2h_gbs, 1), "peak_GBps": round(PCIE5_X16_GBS, 1),
                 "h2d_frac": round(h2d_gbs / PCIE5_X16_GBS, 3),
                 "h2d_bound_Mbps": round(bound, 1), "pinned_frac_of_h2d_bound": round(rate(p_dt) / bound, 3),
                 "measured": "torch pinned->device copies of one batch's samples (x4), device->pinned of its "
                             "payload slots (x4), HIP events"},
        "bit_exact_check": {"pinned": p_ok, "pageable": g_ok, "pageable_registered": r_ok,
                            "checked": f"every packet of all {nb} batches: CRC pass and payload = sent"},
        "host": dict(host, threads_available=threads),
    }), flush=True)


def bench_capture(args):
    """BASELINE config 1: the recorded over-the-air packet of code/WiFi/tests/test_real_rx
    (committed as data in tests/golden/ref_fe.npz) through receiver() -- removeDC, CCA,
    LTS, DataSymbol, FFT, ChannelEqualization, PilotTrack, decode -- batched over captures:
    capture 0 is the KAT stream itself (checked against its ground output), the others the
    same recording with fresh noise, gains and idle lengths."""
    import numpy as np
    from oracle import oracle as O
    from tests import fe_cases
    dev = torch.device("cuda", 0)
    fe = np.load(os.path.join(ROOT, "tests", "golden", "ref_fe.npz"))
    n = args.npkts if args.npkts != 16384 else 4096
    rng = np.random.default_rng(0xC0F1)
    _, real = fe_cases.kat_streams(fe)
    caps = [real]
    for i in range(1, n):
        g = rng.uniform(0.7, 1.5)
        idle = int(rng.integers(340, 1000))
        sig = np.concatenate([np.zeros((idle, 2)), real[1000:].astype(np.float64) * g])
        sig += rng.normal(0, 1.0, sig.shape)
        caps.append(np.clip(np.rint(sig), -32768, 32767).astype(np.int16))
    off = np.cumsum([0] + [c.shape[0] for c in caps]).astype(np.int64)
    x = torch.from_numpy(np.concatenate(caps)).to(dev)
    coff = torch.from_numpy(off[:-1]).to(dev)
    clen = torch.from_numpy(np.diff(off).astype(np.int32)).to(dev)
    max_len = int(np.diff(off).max())
    eng = RxEngine(0)
    payload = torch.zeros((n, 4096), dtype=torch.uint8, device=dev)
    info = torch.zeros((n, 8), dtype=torch.int32, device=dev)
    det = torch.zeros((n, 8), dtype=torch.int32, device=dev)
    step = lambda: eng.rx_stream(x, coff, clen, max_len, False, payload, info, det)
    elapsed = _timed(step, args.steps, args.warmup)
    inf, pay, dt = info.cpu().numpy(), payload.cpu().numpy(), det.cpu().numpy()
    ok = (inf[:, 4] == 1) & (dt[:, 0] == 1)
    bits = int(((inf[:, 2] - 4) * 8 * ok).sum())
    kat = fe["real_out"]
    kat_ok = bool(ok[0] and (pay[0, :kat.size] == kat).all())
    sample = min(64, n)
    cpu_ok = 0
    match = True
    for i in range(sample):                              # parity sample: the oracle, capture by capture
        opay, r, odet, _, _ = O.rx_stream(caps[i])
        if r["ret"] == 0 and r["crc_ok"]:
            cpu_ok += 1
            match &= bool((pay[i, :r["len"] - 4] == opay).all())

    def one(i):                                          # CRC-checked payload bits of capture i
        _, r, _, _, _ = O.rx_stream(caps[i])
        return (r["len"] - 4) * 8 if r["ret"] == 0 and r["crc_ok"] else 0
    threads, host = host_cpus()
    done, cpu_bits, cpu_dt = threaded_baseline(one, n, args.cpu_seconds, threads)
    print(json.dumps({
        "metric": "decoded Mbit/s, recorded 802.11a packet through the full receiver (BASELINE config 1)",
        "value": round(bits * args.steps / elapsed / 1e6, 2), "unit": "Mbit/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int16+int32",
        "data": "recorded capture (test_real_rx.infile) + noise/gain/idle variants",
        "config": {"workload": f"config1: {n} captures of {max_len} samples max, receiver() per capture",
                   "captures_per_s": round(n * args.steps / elapsed, 1)},
        "bit_exact_check": {"kat_capture_matches_ground": kat_ok, "crc_pass": int(ok.sum()),
                            "oracle_sample_match": match, "oracle_sample_crc_pass": cpu_ok},
        "cpu_baseline": {"value": round(cpu_bits / cpu_dt / 1e6, 3), "unit": "Mbit/s", "cores": threads,
                         "kind": "port", "host": host,
                         "sample": f"{done} captures of the batch, {cpu_dt:.1f} s wall on {threads} threads "
                                   "(scalar C oracle receiver(), one capture per call, calls in parallel)"},
    }), flush=True)


def bench_tx(args):
    """transmitter() over config-3 packets (54 Mbps, 1500-byte payloads): header + payload
    bytes in HBM -> 40 MHz samples in HBM; checked against the oracle on a sample."""
    import numpy as np
    from oracle import oracle as O
    dev = torch.device("cuda", 0)
    n, L = args.npkts, args.payload
    rng = np.random.default_rng(0x7E57)
    hdr = O.plcp_header(3, 2, L + 4)
    pk = np.concatenate([np.tile(hdr, (n, 1)), rng.integers(0, 256, (n, L)).astype(np.uint8)], 1)
    per = int(zlib().zrx_tx_samples(hdr.ctypes.data_as(C.c_void_p)))
    d_in = torch.from_numpy(pk.reshape(-1)).to(dev)
    d_ioff = torch.arange(n, dtype=torch.int64, device=dev) * (L + 3)
    d_ooff = torch.arange(n, dtype=torch.int64, device=dev) * per
    d_out = torch.zeros((n * per, 2), dtype=torch.int16, device=dev)
    d_ns = torch.zeros(n, dtype=torch.int32, device=dev)
    eng = RxEngine(0)
    P = lambda t: C.c_void_p(t.data_ptr())

    def step():
        eng._stream()
        rc = zlib().zrx_tx_dev(eng._h, P(d_in), P(d_ioff), n, P(d_out), P(d_ooff), P(d_ns))
        assert rc == 0, rc

    elapsed = _timed(step, args.steps, args.warmup)
    out = d_out.cpu().numpy()
    sample = min(32, n)
    match = all((out[i * per:(i + 1) * per] == O.tx_packet(pk[i])).all() for i in range(sample))
    threads, host = host_cpus()
    done, cpu_bits, cpu_dt = threaded_baseline(lambda i: (O.tx_packet(pk[i]), L * 8)[1], n, args.cpu_seconds, threads)
    bits = n * L * 8
    print(json.dumps({
        "metric": "transmitted payload Mbit/s, 802.11a TX chain at 40 MHz (SURVEY §8f row 4)",
        "value": round(bits * args.steps / elapsed / 1e6, 1), "unit": "Mbit/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int16",
        "data": "synthetic payloads", "config": {"workload": f"tx: {n} packets x {L} B @ 54 Mbps, {per} samples each",
                                                 "gsamples_per_s": round(n * per * args.steps / elapsed / 1e9, 2)},
        "bit_exact_check": {"oracle_sample_match": bool(match), "sample": sample},
        "cpu_baseline": {"value": round(cpu_bits / cpu_dt / 1e6, 2), "unit": "Mbit/s", "cores": threads,
                         "kind": "port", "host": host,
                         "sample": f"{done} packets of the batch, {cpu_dt:.1f} s wall on {threads} threads "
                                   "(scalar C oracle transmitter(), one packet per call, calls in parallel)"},
    }), flush=True)


def threaded_baseline(fn, n, seconds, threads):
    """Runs fn(i) for items i = 0, 1, ... (mod n) on `threads` Python threads (the oracle's
    ctypes calls release the GIL) until `seconds` of wall time have passed; returns (items
    done, sum of fn's results, seconds)."""
    import concurrent.futures as cf
    import itertools
    done = total = 0
    ctr = itertools.count()
    t0 = time.perf_counter()

    def worker():
        k = s = 0
        while time.perf_counter() - t0 < seconds or k == 0:
            s += fn(next(ctr) % n)
            k += 1
        return k, s
    with cf.ThreadPoolExecutor(max_workers=threads) as ex:
        for k, s in ex.map(lambda _: worker(), range(threads)):
            done += k
            total += s
    return done, total, time.perf_counter() - t0


def host_cpus():
    """(threads to use, description) for the CPU baseline: every core this process may run
    on (sched_getaffinity), capped by the cgroup CPU quota (cpu.max) and OMP_NUM_THREADS
    when those are set (the GPU box gives one GPU's job a 16-core share), plus the CPU
    model string."""
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    omp = int(os.environ["OMP_NUM_THREADS"]) if os.environ.get("OMP_NUM_THREADS", "").isdigit() else None
    threads = min(x for x in (aff, quota, omp) if x)
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return threads, {"nproc": nproc, "affinity": aff, "cgroup_cpu_quota": quota, "omp_num_threads": omp,
                     "cpu_model": model}


def cpu_baseline(b, seconds, chan=None):
    """The chain on every host core this process is allowed (host_cpus), packet-parallel with
    pthreads, over chunks of the same packets until `seconds` of wall time have passed: the
    fast CPU port (oracle/cpu_port.c: table FFT, AVX-512 Viterbi, table CRC; bit-identical to
    the oracle, tests/test_cpu_port.py), with ChannelEqualization + PilotTrack for the EQ
    chain."""
    from oracle import oracle as O
    threads, host = host_cpus()
    sym = b["sym"].cpu().numpy()
    off_all = b["sym_off"].cpu().numpy()
    ns_all = b["nsym"].cpu().numpy()
    ch_all = chan.cpu().numpy() if chan is not None else None
    chunk = max(1024, 64 * threads)
    done = ok = bits = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        lo = done % off_all.size
        hi = min(lo + chunk, off_all.size)
        if ch_all is None:
            _, res = O.rx_batch_time_fast(sym, off_all[lo:hi], ns_all[lo:hi], nthreads=threads)
        else:
            _, res = O.rx_batch_time_eq_fast(sym, off_all[lo:hi], ns_all[lo:hi], ch_all[lo:hi], nthreads=threads)
        ok += sum(r["crc_ok"] for r in res)
        bits += sum((r["len"] - 4) * 8 for r in res if r["crc_ok"])
        done += hi - lo
    dt = time.perf_counter() - t0
    fast = O.rx_batch_time_eq_fast if ch_all is not None else O.rx_batch_time_fast
    what = "CPU port: table FFT, %s%s Viterbi, table CRC" % (
        "the oracle's ChannelEqualization + PilotTrack, " if ch_all is not None else "",
        "AVX-512 vpermb" if getattr(fast, "avx512", False) else "scalar")
    return {"value": round(bits / dt / 1e6, 2), "unit": "Mbit/s", "cores": threads, "kind": "port",
            "per_core": round(bits / dt / 1e6 / threads, 2), "host": host,
            "sample": f"{done} packets of the same batch ({ok} CRC-ok), {dt:.1f} s wall on {threads} threads "
                      f"({what}; the reference SSE2 Viterbi brick alone runs 41-73 Mbit/s per core, SURVEY.md §6)"}


if __name__ == "__main__":
    main()
