"""Host logic of the node behind the batched externals (ziria_amd/csrc/zrx_shard.hpp): how a
call is split into contiguous packet ranges over the GPUs of a node and how the ranges'
results merge (no GPU: zrx_shard_split / zrx_shard_selftest run on the host; the GPU tests
in test_gpu_node.py drive the same code with real shards)."""
import ctypes as C

import numpy as np
import pytest

from ziria_amd._lib import lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _split(prefix, nshards, min_bytes=0):
    prefix = np.ascontiguousarray(prefix, np.int64)
    cut = np.zeros(nshards + 2, np.int32)
    k = lib().zrx_shard_split(_p(prefix), prefix.size - 1, nshards, min_bytes, _p(cut))
    assert k >= 1
    return cut[:k + 1]


def _weights(rng, n, kind):
    if kind == "uniform":
        return np.full(n, 57 * 256, np.int64)                      # config 3: 57 symbols a packet
    if kind == "mixed":                                            # config 5: 64..4095 B at 6..54 Mbps
        return rng.integers(3, 700, n).astype(np.int64) * 256
    if kind == "skewed":                                           # a few huge packets among small ones
        w = rng.integers(1, 10, n).astype(np.int64) * 256
        w[rng.integers(0, n, max(1, n // 50))] *= 400
        return w
    if kind == "zeros":
        w = np.zeros(n, np.int64)
        return w
    raise ValueError(kind)


@pytest.mark.parametrize("nshards", range(1, 9))
@pytest.mark.parametrize("kind", ["uniform", "mixed", "skewed", "zeros"])
def test_split_contiguous_balanced(nshards, kind):
    rng = np.random.default_rng(nshards * 31 + len(kind))
    for n in (1, 2, 7, nshards, 1000, 16384):
        w = _weights(rng, n, kind)
        prefix = np.concatenate([[1000], 1000 + np.cumsum(w)])   # (a base offset: prefixes need not start at 0)
        cut = _split(prefix, nshards)
        k = cut.size - 1
        assert cut[0] == 0 and cut[-1] == n and (np.diff(cut) > 0).all()   # every packet once, in order, no empty range
        assert k == min(nshards, n)
        total, per = int(w.sum()), [int(w[cut[j]:cut[j + 1]].sum()) for j in range(k)]
        if total:
            # no range carries more than its share plus one packet
            assert max(per) <= -(-total // k) + int(w.max()), (per, total)
        else:
            assert max(np.diff(cut)) - min(np.diff(cut)) <= 1


def test_split_min_bytes():
    w = np.full(16384, 57 * 256, np.int64)                         # 239 MB of config-3 symbols
    prefix = np.concatenate([[0], np.cumsum(w)])
    assert _split(prefix, 8, 16 << 20).size - 1 == 8
    assert _split(prefix, 8, 100 << 20).size - 1 == 2              # 239 MB / 100 MB
    assert _split(prefix[:11], 8, 16 << 20).size - 1 == 1          # 10 packets: one shard
    assert _split(prefix[:11], 8, 0).size - 1 == 8                 # forced onto every shard


def test_split_rejects_bad_prefix():
    prefix = np.array([0, 5, 3], np.int64)
    cut = np.zeros(4, np.int32)
    assert lib().zrx_shard_split(_p(prefix), 2, 2, 0, _p(cut)) == -1
    assert lib().zrx_shard_split(_p(prefix), 2, 0, 0, _p(cut)) == -1


@pytest.mark.parametrize("nshards", range(1, 9))
def test_runner_merges_ranges(nshards):
    """The shard runner's merge: each range (one thread each) writes only its own packets into
    the caller's array, and the call returns the sum of their counts."""
    rng = np.random.default_rng(nshards)
    w = _weights(rng, 3000, "mixed")
    prefix = np.ascontiguousarray(np.concatenate([[0], np.cumsum(w)]), np.int64)
    owner = np.full(3000, -1, np.int32)
    rc = lib().zrx_shard_selftest(_p(prefix), 3000, nshards, 0, _p(owner), -1)
    assert rc == 3000
    cut = _split(prefix, nshards)
    expect = np.repeat(np.arange(cut.size - 1), np.diff(cut))
    assert (owner == expect).all()


def test_runner_reports_first_failing_range():
    w = np.full(100, 256, np.int64)
    prefix = np.ascontiguousarray(np.concatenate([[0], np.cumsum(w)]), np.int64)
    owner = np.full(100, -1, np.int32)
    assert lib().zrx_shard_selftest(_p(prefix), 100, 4, 0, _p(owner), 2) == -6     # ZRX_EINTERNAL
    # the other ranges still ran to completion (every thread has returned when the call does)
    cut = _split(prefix, 4)
    for j in (0, 1, 3):
        assert (owner[cut[j]:cut[j + 1]] == j).all()
    assert (owner[cut[2]:cut[3]] == -1).all()


def test_node_without_gpu_fails_loudly():
    """No gfx950 device here: the node has no shards and the batched externals refuse."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    devs = np.zeros(8, np.int32)
    assert lib().zrx_get_devices(_p(devs), 8) == -4                # ZRX_ENODEV
    one = np.array([0], np.int32)
    assert lib().zrx_set_devices(_p(one), 1, -1) == -4
    assert lib().zrx_set_devices(None, 0, -1) == 0                 # (the default list: resolved at first use)
    st = np.zeros(8, np.int64)
    assert lib().zrx_node_stats(_p(st)) == 0 and st[7] == 16 << 20
