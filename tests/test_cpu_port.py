"""The fast CPU port (oracle/cpu_port.c, bench.py's cpu_baseline leg) gives the oracle's
results packet for packet: clean, mixed-MCS, CRC-failing, truncated and bad-header packets."""
import ctypes

import numpy as np

from ziria_amd import txgen


def _same(oracle, sym, off, ns):
    p1, r1 = oracle.rx_batch_time(sym, off, ns, nthreads=8)
    p2, r2 = oracle.rx_batch_time_fast(sym, off, ns, nthreads=8)
    assert r1 == r2
    assert (p1 == p2).all()
    return r2


def test_port_54mbps_and_noise_edge(oracle):
    for seed, sigma in ((3, 4.0), (9, 58.0)):
        b = txgen.make_batch(96, seed=seed, sigma=sigma)
        r = _same(oracle, b["sym"].numpy(), b["sym_off"].numpy(), b["nsym"].numpy())
        assert sum(x["crc_ok"] for x in r) > 10


def test_port_mixed_mcs(oracle):
    m = txgen.make_mixed(128, max_len=2300, sigma=3.0, seed=21)
    r = _same(oracle, m["sym"].numpy(), m["sym_off"].numpy(), m["nsym"].numpy())
    assert len({(x["modulation"], x["coding"]) for x in r}) == 8


def test_port_truncated_and_bad_header(oracle):
    b = txgen.make_batch(8, seed=4)
    sym = b["sym"].numpy().copy()
    ns = b["nsym"].numpy().copy()
    ns[1] = 10
    S = b["max_nsym"]
    sym[2 * S] = 0
    _same(oracle, sym, b["sym_off"].numpy(), ns)


def test_port_fft64_vs_oracle(oracle):
    rng = np.random.default_rng(5)
    x = rng.integers(-32768, 32768, size=(3000, 64, 2), dtype=np.int16)
    x[:500] = rng.choice(np.array([-32768, 32767, -1, 0], np.int16), size=(500, 64, 2))
    x[500:1000] >>= 6
    got = np.zeros_like(x)
    L = oracle.lib()
    L.zp_fft64.restype = ctypes.c_int
    L.zp_fft64(oracle._p(x), oracle._p(got), x.shape[0])
    want = oracle.fft64(x.reshape(-1, 64, 2))
    assert (got == want.reshape(got.shape)).all()


def test_port_viterbi_batch_vs_oracle(oracle):
    """zp_viterbi_batch (config 2's CPU baseline) equals zo_viterbi_batch: all rates, lengths
    1..4095 B, clean to pure-noise soft values, truncated input."""
    from tests.golden import synth
    rng = np.random.default_rng(31)
    softs, fl, cr = [], [], []
    for i in range(60):
        c = i % 3
        f = int(rng.choice([1, 3, 100, 1500, 4095])) if i % 5 else int(rng.integers(1, 2048))
        s = synth.viterbi_soft(c, f, int(rng.integers(-1, 6)), seed=400 + i)
        if i % 7 == 6:
            s = s[: s.size // 2 // 12 * 12]
        softs.append(s); fl.append(f); cr.append(c)
    sl = np.array([s.size for s in softs], np.int64)
    so = np.cumsum(sl) - sl
    oo = np.cumsum(np.array(fl, np.int64) + 16) - (np.array(fl, np.int64) + 16)
    size = int(oo[-1] + fl[-1] + 16)
    args = (np.concatenate(softs), so, sl, fl, cr, oo, size)
    a = oracle.viterbi_batch(*args, nthreads=4)
    b = oracle.viterbi_batch(*args, nthreads=4, fast=True)
    assert (a == b).all()


def test_port_eq_chain_vs_oracle(oracle, golden):
    """the port's EQ chain (bench.py --eq cpu_baseline) equals the oracle's: the reference
    fixture's packets and a synthetic channel batch at two noise levels"""
    eq = golden["ref_eq"]
    args = (eq["eq_sym"], eq["eq_off"], eq["eq_nsym"], eq["eq_chan"])
    p1, r1 = oracle.rx_batch_time_eq(*args, nthreads=4)
    p2, r2 = oracle.rx_batch_time_eq_fast(*args, nthreads=4)
    assert r1 == r2 and (p1 == p2).all()
    for seed, sigma in ((5, 2.0), (6, 40.0)):
        b = txgen.make_batch(64, seed=seed, sigma=sigma, channel=True)
        a = (b["sym"].numpy(), b["sym_off"].numpy(), b["nsym"].numpy(), b["chan"].numpy())
        p1, r1 = oracle.rx_batch_time_eq(*a, nthreads=8)
        p2, r2 = oracle.rx_batch_time_eq_fast(*a, nthreads=8)
        assert r1 == r2 and (p1 == p2).all()
        if sigma < 10:
            assert sum(x["crc_ok"] for x in r2) > 32
