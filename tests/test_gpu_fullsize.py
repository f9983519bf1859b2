"""Packet-for-packet parity at BASELINE's full batch sizes: every one of 16384 packets of a
config-3 batch (clean, and at the noise edge where CRCs fail), and of a 16384-packet config-5
batch of distinct mixed-MCS packets, decoded by the HIP chain, against the same batch decoded
on the host by oracle/cpu_port.c.  The port is the oracle's chain written for speed, identical
to the oracle (tests/test_cpu_port.py), so it can check a whole batch in about a second; the
oracle itself checks the smaller GPU cases in test_gpu_parity.py."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from ziria_amd import txgen  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402


def _threads():
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return 8


def _check(oracle, b):
    n = b["sym_off"].numel()
    chan = b.get("chan")
    e = RxEngine(0)
    try:
        e.reserve(n, b["max_nsym"])
        pay, info = e.rx(b["sym"], b["sym_off"], b["nsym"], b["max_nsym"], chan=chan)
        torch.cuda.synchronize()
        pay, info = pay.cpu().numpy(), info.cpu().numpy()
    finally:
        e.close()
    args = (b["sym"].cpu().numpy(), b["sym_off"].cpu().numpy(), b["nsym"].cpu().numpy())
    if chan is None:
        opay, res = oracle.rx_batch_time_fast(*args, nthreads=_threads())
    else:
        opay, res = oracle.rx_batch_time_eq_fast(*args, chan.cpu().numpy(), nthreads=_threads())
    hdr = np.array([(r["modulation"], r["coding"], r["len"], r["err"]) for r in res], np.int32)
    crc = np.array([r["crc_ok"] for r in res], np.int32)
    assert (info[:, :4] == hdr).all(), np.nonzero((info[:, :4] != hdr).any(1))[0][:10]
    assert (info[:, 4] == crc).all(), np.nonzero(info[:, 4] != crc)[0][:10]
    plen = np.maximum(hdr[:, 2] - 4, 0)
    bad = [i for i in range(n) if not hdr[i, 3] and not (pay[i, :plen[i]] == opay[i, :plen[i]]).all()]
    assert not bad, bad[:10]
    return crc, pay


def test_fullsize_config3_vs_port(oracle):
    b = txgen.make_batch(16384, seed=0x5EED, sigma=4.0, device="cuda")
    crc, _ = _check(oracle, b)
    assert crc.all()


def test_fullsize_config3_noise_edge_vs_port(oracle):
    b = txgen.make_batch(16384, seed=58, sigma=58.0, device="cuda")
    crc, _ = _check(oracle, b)
    assert 0 < crc.sum() < crc.size                        # CRC failures do occur here


def test_fullsize_config5_vs_port(oracle):
    m = txgen.make_mixed_fast(16384, min_len=64, max_len=4095, sigma=3.0, seed=0xC5C6, device="cuda")
    crc, _ = _check(oracle, m)
    assert crc.sum() > 7000


@pytest.mark.parametrize("seed", [0x5EED, 0x5EEE])
def test_fullsize_eq_bench_batches_vs_port(oracle, seed):
    """The exact batches of `bench.py --eq` (FFT >>> ChannelEqualization >>> PilotTrack >>>
    GetData, 3-tap channel + phase drift, AWGN sigma 2; seeds 0x5EED / 0x5EEE): header, CRC
    verdict and payload of all 16384 packets against the port's EQ chain.  Some packets fail
    their CRC at this noise level; every CRC-passing one must carry what was sent."""
    b = txgen.make_batch_range(0, 16384, mod=3, coding=2, payload_len=1500, sigma=2.0, seed=seed,
                               device="cuda", channel=True)
    crc, pay = _check(oracle, b)
    ok = crc == 1
    assert 16000 < ok.sum() < 16384
    assert (pay[ok, :1500] == b["payload"][ok]).all()


def test_mixed_noise_frames_vs_port(oracle):
    """A mixed batch with every fourth packet's data symbols replaced by noise: those frames
    decode to garbage, their segments' warm-ups need not converge, and the seam pass
    re-decodes from the seams whose two sides disagree.  Every packet against the port, bit
    for bit."""
    m = txgen.make_mixed_fast(4096, min_len=64, max_len=2048, sigma=3.0, seed=0x5EA4, device="cuda")
    sym = m["sym"].clone()
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    off, ns = m["sym_off"].cpu().numpy(), m["nsym"].cpu().numpy()
    for i in range(0, 4096, 4):
        a, n = int(off[i]) + 1, int(ns[i]) - 1          # (the SIGNAL symbol stays: a valid header)
        if n > 0:
            sym[a:a + n] = torch.randint(-3000, 3000, (n, 64, 2), generator=g, device="cuda", dtype=torch.int16)
    b = dict(m, sym=sym)
    e = RxEngine(0)
    e.reserve(4096, m["max_nsym"])
    e.rx(sym, m["sym_off"], m["nsym"], m["max_nsym"])
    torch.cuda.synchronize()
    rows, fixes = e.plan_stats()
    e.close()
    crc, _ = _check(oracle, b)
    print(f"crc pass {crc.sum()} of 4096, rows {rows}, seam fixes {fixes}")
    assert 2000 < crc.sum() < 3200
