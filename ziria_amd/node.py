"""Packet sharding across the GPUs of one node.

Packets are independent, so a batch is split into contiguous packet ranges, one per rank,
and decoded with no collective in the hot loop.  After decoding, one exchange over
torch.distributed (RCCL over xGMI on the GPU node; gloo in the CPU tests) combines the
per-rank results: a sum of {CRC-pass count, payload bits, bit-exact flags} and a gather of
the decoded payload bytes to the destination rank.  The reference has no distributed code
(its only parallelism is intra-process pipeline threading, src/Pipeline/PassPipeline.hs:144),
so this is new, and it never changes per-packet results.
"""
import torch
import torch.distributed as dist


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


def combine(ok, bits, match, payload=None, dst=0, device=None):
    """Sums the per-rank counts over the default process group and gathers `payload`
    ([n, L] uint8, the same shape on every rank) to `dst`.  Returns
    (ok_total, bits_total, ranks_matching, gathered list or None)."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    t = torch.tensor([ok, bits, match], dtype=torch.int64, device=device)
    if world == 1:
        return ok, bits, match, ([payload] if payload is not None else None)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    gathered = None
    if payload is not None:
        rank = dist.get_rank()
        gathered = [torch.empty_like(payload) for _ in range(world)] if rank == dst else None
        dist.gather(payload, gathered, dst=dst)
    o, b, m = (int(v) for v in t.tolist())
    return o, b, m, gathered


def max_over_ranks(seconds, device=None):
    """The slowest rank's elapsed time (the bench's timing rule)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
