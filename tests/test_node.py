"""The N>1 path of bench.py (ziria_amd/node.py) on CPU: world_size-2 gloo process groups
stand in for RCCL.  Per-rank decode results come from a stub decoder here (the decode itself
is GPU-only); what is checked is the sharding, the timed loop, the final combine of counts
and the gather + per-packet check of payloads, including unequal shards.  run_sharded is
the function bench.py's main() calls, so this is the driver's 1/2/4/8-GPU code path."""
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
            out.put((o, b, m, elapsed, g.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,npkts", [(2, 10), (2, 11), (3, 7)])
def test_combine_over_gloo(world, npkts):
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


L = 24


def _payload(lo, hi, b=0):
    return ((torch.arange(lo, hi).unsqueeze(1) * 7 + torch.arange(L) + 13 * b) % 251).to(torch.uint8).numpy()


def _bench_worker(rank, world, port, total, corrupt, out):
    """bench.py main() with the engine replaced by a stub that 'decodes' by copying the
    transmitted payload (and, with corrupt, flips one byte of global packet 5)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = {"step": [], "verify": []}

        def make_shard(lo, hi):
            return {"lo": lo, "hi": hi, "pay": torch.zeros((hi - lo, 64), dtype=torch.uint8),
                    "info": torch.zeros((hi - lo, 8), dtype=torch.int32)}

        def decode(sh, b):
            sh["pay"][:, :L] = torch.from_numpy(_payload(sh["lo"], sh["hi"], b))
            if corrupt and b == 1 and sh["lo"] <= 5 < sh["hi"]:
                sh["pay"][5 - sh["lo"], 3] ^= 1
            sh["info"][:, 2] = L + 4
            sh["info"][:, 4] = 1

        def step(sh, k):
            calls["step"].append(k)
            decode(sh, k % 2)

        def outputs(sh, b):
            calls["verify"].append(b)
            decode(sh, b)
            return sh["pay"], sh["info"]

        timed = []
        res = node.run_sharded(total, make_shard, step, outputs, _payload,
                               steps=3, warmup=2, payload_len=L, on_timed=timed.append, nbatches=2)
        out.put((rank, res["lo"], res["hi"], calls, timed, res["ok"], res["bits"],
                 res.get("packets"), res.get("payload_match"), res.get("mismatched_packets")))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total,corrupt", [(2, 11, False), (2, 16, False), (2, 11, True), (3, 11, False)])
def test_run_sharded_over_gloo(world, total, corrupt):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, total, corrupt, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ranges = [(g[1], g[2]) for g in got]
    assert ranges == [node.shard_range(total, world, r) for r in range(world)]
    for g in got:
        assert g[3] == {"step": [0, 1, 2, 3, 4], "verify": [0, 1]}   # 2 warmup + 3 timed steps, both batches checked
        assert g[4] == [True, False]                                # timers on / off
        assert g[5] == 2 * total and g[6] == total * L * 8          # summed over ranks (CRC passes of both batches)
    r0 = got[0]
    assert r0[7] == 2 * total
    assert r0[8] is (not corrupt)
    assert r0[9] == (1 if corrupt else 0)


def test_run_sharded_single_process():
    res = node.run_sharded(5, lambda lo, hi: {"p": torch.from_numpy(_payload(lo, hi)),
                                              "i": torch.ones((hi - lo, 8), dtype=torch.int32) * 0 + torch.tensor([0, 0, L + 4, 0, 1, 0, 0, 0], dtype=torch.int32)},
                           lambda sh, k: None, lambda sh, b: (sh["p"], sh["i"]), _payload, steps=1, warmup=0,
                           payload_len=L)
    assert (res["lo"], res["hi"], res["ok"], res["packets"], res["payload_match"]) == (0, 5, 5, 5, True)


def test_run_sharded_batches_keep_their_own_info():
    """outputs() returns the decoder's live buffers (as bench.py's engine does), so batch 1's
    decode overwrites batch 0's info; each batch's payload must still be judged against its
    own CRC flags.  Batch 0 fails the CRC of packet 2 and leaves garbage there (a CRC-failing
    packet's payload is not checked with crc_ok_only), batch 1 passes every packet."""
    live = {"p": torch.zeros((5, 64), dtype=torch.uint8), "i": torch.zeros((5, 8), dtype=torch.int32)}

    def decode(b):
        live["p"][:, :L] = torch.from_numpy(_payload(0, 5, b))
        live["i"][:, 2] = L + 4
        live["i"][:, 4] = 1
        if b == 0:
            live["p"][2, :L] ^= 0x5A
            live["i"][2, 4] = 0

    def outputs(sh, b):
        decode(b)
        return live["p"], live["i"]

    res = node.run_sharded(5, lambda lo, hi: live, lambda sh, k: decode(k % 2), outputs, _payload, steps=2,
                           warmup=1, payload_len=L, crc_ok_only=True, nbatches=2)
    assert res["ok"] == 9 and res["packets"] == 10
    assert res["payload_match"] is True and res["mismatched_packets"] == 0
    assert res["bits_per_batch"] == [4 * L * 8, 5 * L * 8]
