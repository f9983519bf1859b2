"""Packet sharding across the GPUs of one node (BASELINE config 4).

Packets are independent, so a batch is split into contiguous packet ranges, one per rank,
and decoded with no collective in the hot loop.  After decoding, one exchange over
torch.distributed (RCCL over xGMI on the GPU node; gloo in the CPU tests) combines the
per-rank results: a sum of {CRC-pass count, payload bits, bit-exact flags} and a gather of
the decoded payload bytes and packet infos to the destination rank, where every packet is
checked against what was transmitted.  The reference has no distributed code (its only
parallelism is intra-process pipeline threading, src/Pipeline/PassPipeline.hs:144), so this
is new, and it never changes per-packet results.

`run_sharded` is the whole N-rank bench step loop (bench.py drives it with the HIP engine,
tests/test_node.py with a stub decoder over gloo), so the path the driver's 1/2/4/8-GPU
runs take is the path the CPU tests cover.
"""
import time

import numpy as np
import torch
import torch.distributed as dist


def world_rank():
    if dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def comm_device(device=None):
    """Where collective tensors live: the GPU for RCCL ("nccl"), the host for gloo (the CPU
    tests, and bench.py --share-gpu, where the ranks share one GPU)."""
    if dist.is_initialized() and dist.get_backend() == "gloo":
        return torch.device("cpu")
    return device


def shard_range(npkts, world, rank):
    """Contiguous [start, stop) packet range of `rank`; sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world or npkts < 0:
        raise ValueError(f"bad shard request npkts={npkts} world={world} rank={rank}")
    base, extra = divmod(npkts, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def counts(info, payload_len=None, payload=None, expected=None, crc_ok_only=False):
    """Per-rank totals from an info tensor [n, 8] (ziria_rx.h layout): CRC-pass count,
    CRC-checked payload bits, and 1 if `payload` equals `expected` (when given; on the
    CRC-passing packets only with crc_ok_only)."""
    crc_ok = info[:, 4] == 1
    ok = int(crc_ok.sum())
    bits = int(((info[:, 2].to(torch.int64) - 4) * 8 * crc_ok).sum())
    match = 1
    if expected is not None:
        exp = torch.as_tensor(expected, device=payload.device)
        eq = payload[:, :exp.shape[1]] == exp
        match = int(bool(eq[crc_ok].all() if crc_ok_only else eq.all()))
    return ok, bits, match


def gather_rows(t, dst=0):
    """Gathers a [n_r, ...] tensor from every rank to `dst`, where n_r may differ per rank
    (unequal shards): each rank pads to the largest n_r, the padded blocks are gathered,
    and `dst` trims them.  Returns the row-wise concatenation in rank order on `dst`
    (the tensor itself with one rank), None elsewhere."""
    world, rank = world_rank()
    if world == 1:
        return t
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    cap = max(sizes)
    pad = torch.zeros((cap,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[:t.shape[0]] = t
    blocks = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
    dist.gather(pad, blocks, dst=dst)
    if rank != dst:
        return None
    return torch.cat([b[:s] for b, s in zip(blocks, sizes)], 0)


def combine(ok, bits, match, payload=None, dst=0, device=None):
    """Sums the per-rank counts over the default process group and gathers `payload`
    ([n_r, L] uint8; n_r may differ per rank) to `dst`.  Returns (ok_total, bits_total,
    ranks_matching, gathered payload rows on dst or None)."""
    world, _ = world_rank()
    if world == 1:
        return ok, bits, match, payload
    t = torch.tensor([ok, bits, match], dtype=torch.int64, device=comm_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    gathered = gather_rows(payload, dst) if payload is not None else None
    o, b, m = (int(v) for v in t.tolist())
    return o, b, m, gathered


def max_over_ranks(seconds, device=None):
    """The slowest rank's elapsed time (the bench's timing rule)."""
    world, _ = world_rank()
    if world == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=comm_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_floats(values, device=None):
    """Every rank's list of floats (same length on every rank), in rank order."""
    world, _ = world_rank()
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=comm_device(device))
    if world == 1:
        return [t.tolist()]
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def barrier(device=None):
    if world_rank()[0] > 1:
        dist.barrier()


def _sync(device):
    if device is not None and device.type == "cuda":
        torch.cuda.synchronize(device)


def run_sharded(total, make_shard, step, outputs, expected, steps, warmup, payload_len, device=None,
                crc_ok_only=False, on_timed=None, nbatches=1, on_step=None):
    """The bench's N-rank loop over one global batch of `total` packets.

    make_shard(lo, hi) builds this rank's packets [lo, hi) (already in device memory) as
    `nbatches` distinct batches of the same shape (a streaming receiver never decodes the same
    samples twice, so the timed steps rotate through them); step(shard, k) runs decode step k
    (k counts from 0 over the warmup and timed steps: bench.py decodes batch k % nbatches);
    outputs(shard, b) -> (payload uint8 [n, >=L], info int32 [n, 8]) of batch b, decoded once
    more after the timed region; expected(lo, hi, b) -> uint8 numpy [hi-lo, L], the
    transmitted payloads of batch b (L = payload_len bytes each), which rank 0 uses to check
    every gathered packet of every batch.
    on_timed(True) is called after the warmup, before the barrier that opens the timed region
    (bench.py runs its instrumented stage-timer pass there), on_timed(False) after it closes.
    on_step(i), when given, is called at the start of the timed region (i = -1) and after each
    timed step i (bench.py records a HIP event there: per-step times).

    Timing: `warmup` untimed steps, then barrier + device sync, `steps` timed steps, device
    sync + barrier, and the slowest rank's time.  Returns on every rank a dict with the
    shard, the timing and the combined counts (`bits` = CRC-checked payload bits per timed
    step, all ranks: the mean over the batches the timed steps decoded); rank 0's also holds
    the per-packet check over all batches."""
    world, rank = world_rank()
    lo, hi = shard_range(total, world, rank)
    shard = make_shard(lo, hi)
    k = 0
    for _ in range(warmup):
        step(shard, k)
        k += 1
    _sync(device)
    if on_timed:
        on_timed(True)
    _sync(device)
    barrier(device)
    _sync(device)
    t0 = time.perf_counter()
    if on_step:
        on_step(-1)
    timed_batches = []
    for i in range(steps):
        step(shard, k)
        if on_step:
            on_step(i)
        timed_batches.append(k % nbatches)
        k += 1
    _sync(device)
    t_own = time.perf_counter() - t0                 # this rank's own time (before the closing barrier)
    barrier(device)
    t1 = time.perf_counter()
    if on_timed:
        on_timed(False)
    elapsed = max_over_ranks(t1 - t0, device=device)
    rank_elapsed = [r[0] for r in all_gather_floats([t_own], device=device)]

    L = payload_len
    ok_b, bits_b, pay_b, info_b = [], [], [], []
    gather_s = 0.0
    for b in range(nbatches):
        payload, info = outputs(shard, b)
        # outputs() may hand back the engine's live buffers, which the next batch's decode
        # overwrites; at world 1 gather_rows returns its argument itself, so keep copies of
        # this batch's rows (the payload slice is a copy already, the info would not be)
        payload, info = payload[:, :L].clone(), info.clone()
        cd = comm_device(device)
        if cd is not None:
            payload, info = payload.to(cd), info.to(cd)
        ok, bits, _ = counts(info)
        _sync(device)
        tg = time.perf_counter()
        ok_all, bits_all, _, pay_all = combine(ok, bits, 1, payload, device=device)
        info_all = gather_rows(info)
        _sync(device)
        gather_s += time.perf_counter() - tg
        ok_b.append(ok_all)
        bits_b.append(bits_all)
        pay_b.append(pay_all)
        info_b.append(info_all)
    bits_per_step = sum(bits_b[b] for b in timed_batches) / max(steps, 1)
    res = dict(lo=lo, hi=hi, shard=shard, elapsed=elapsed, rank_elapsed=rank_elapsed, steps=steps, ok=sum(ok_b),
               bits=bits_per_step,
               bits_per_batch=bits_b, gather_s=gather_s / max(nbatches, 1), world=world, rank=rank, batches=nbatches)
    if rank == 0:
        packets = mism = 0
        match = True
        for b in range(nbatches):
            pay = pay_b[b].cpu().numpy()
            inf = info_b[b].cpu().numpy()
            exp = np.asarray(expected(0, total, b))
            crc = inf[:, 4] == 1
            same = (pay[:, :exp.shape[1]] == exp).all(axis=1)
            packets += int(pay.shape[0])
            match &= bool(same[crc].all() if crc_ok_only else same.all())
            mism += int((~same & (crc if crc_ok_only else True)).sum())
        res["packets"] = packets
        res["payload_match"] = match
        res["mismatched_packets"] = mism
    return res
