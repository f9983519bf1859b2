"""The N>1 path of bench.py (ziria_amd/node.py) on CPU: world_size-2 gloo process groups
stand in for RCCL.  Per-rank decode results are synthetic here (the decode itself is
GPU-only); what is checked is the sharding and the final combine of counts and payloads."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ziria_amd import node


def test_shard_range_covers_exactly():
    for n in (0, 1, 7, 16384, 16385):
        for w in (1, 2, 3, 8):
            rs = [node.shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        node.shard_range(10, 2, 2)


def test_counts_single_rank():
    info = torch.zeros((4, 8), dtype=torch.int32)
    info[:, 2] = 1504
    info[:, 4] = torch.tensor([1, 1, 0, 1], dtype=torch.int32)
    pay = torch.arange(4 * 16, dtype=torch.int64).reshape(4, 16).to(torch.uint8)
    ok, bits, match = node.counts(info, payload=pay, expected=pay[:, :10].numpy())
    assert (ok, bits, match) == (3, 3 * 1500 * 8, 1)
    assert node.combine(ok, bits, match)[:3] == (3, 3 * 1500 * 8, 1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, npkts, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = node.shard_range(npkts, world, rank)
        n = hi - lo
        info = torch.zeros((n, 8), dtype=torch.int32)
        info[:, 2] = 1504
        info[:, 4] = 1
        if rank == 1 and n:
            info[0, 4] = 0                       # one CRC failure on rank 1
        pay = ((torch.arange(lo, hi).unsqueeze(1) * 7 + torch.arange(24)) % 251).to(torch.uint8)
        ok, bits, match = node.counts(info, payload=pay, expected=pay.numpy())
        elapsed = node.max_over_ranks(0.5 + rank)
        o, b, m, g = node.combine(ok, bits, match, pay)
        if rank == 0:
            out.put((o, b, m, elapsed, torch.cat(g).tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_combine_over_gloo(world):
    npkts = 10                                   # equal shards (gather needs equal shapes)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, npkts, q)) for r in range(world)]
    for p in procs:
        p.start()
    o, b, m, elapsed, gathered = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert o == npkts - 1
    assert b == (npkts - 1) * 1500 * 8
    assert m == world
    assert elapsed == 0.5 + (world - 1)
    exp = ((torch.arange(npkts).unsqueeze(1) * 7 + torch.arange(24)) % 251).to(torch.uint8)
    assert gathered == exp.tolist()
