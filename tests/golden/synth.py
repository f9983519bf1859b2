"""Deterministic synthetic inputs for tests and fixture generation (test infrastructure).

* viterbi_soft: BASELINE config 2 recipe — random bits + 6 zero tail, convolutionally
  encoded (code/WiFi/transmitter/encoding.blk), soft = 7*bit + U[-noise, noise] clipped
  to [0, 7], zero-bit extension to a multiple of 48 soft values.
* packets_time: BASELINE config 3/5 recipe — TX via the oracle's
  transmitter restatement, data bins placed in GetData order, x = IDFT(X/100)*64 + N(0,s^2),
  rounded to int16.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

# data-bin order of GetData.blk:24-35
DATA_BINS = np.array(list(range(38, 43)) + list(range(44, 57)) + list(range(58, 64)) +
                     list(range(1, 7)) + list(range(8, 21)) + list(range(22, 27)), np.int64)
PILOT_BINS = np.array([7, 21, 43, 57], np.int64)
BITS_PER_48 = {0: 24, 1: 32, 2: 36}          # input bits per 48 soft values, by code rate


def viterbi_soft(code_rate, frame_len, noise, seed):
    rng = np.random.default_rng(seed)
    need = 8 * frame_len + 6
    K = BITS_PER_48[code_rate]
    n_in = -(-need // K) * K
    bits = np.zeros(n_in, np.uint8)
    bits[: 8 * frame_len] = rng.integers(0, 2, 8 * frame_len)
    coded = O.tx_encode(bits, code_rate).astype(np.int16)
    if noise < 0:
        soft = rng.integers(0, 8, coded.size)
    else:
        soft = np.clip(coded * 7 + rng.integers(-noise, noise + 1, coded.size), 0, 7)
    assert soft.size % 48 == 0
    return soft.astype(np.int8)


def plan_54mbps(n, payload_len):
    return [(3, 2, payload_len)] * n


MCS = [(0, 0), (0, 2), (1, 0), (1, 2), (2, 0), (2, 2), (3, 1), (3, 2)]


def plan_mixed(n, min_len=60, max_len=4091, seed=0x3C5):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        mod, cod = MCS[int(rng.integers(0, 8))]
        out.append((mod, cod, int(rng.integers(min_len, max_len + 1))))
    return out


def packets_time(plan, seed, sigma=4.0, extra_sym=0):
    """Returns (sym int16 [S,64,2], sym_off int64 [n], nsym int32 [n], meta int32 [n,3])."""
    rng = np.random.default_rng(seed)
    syms, offs, nsyms, meta = [], [], [], []
    off = 0
    for (mod, cod, plen) in plan:
        pay = rng.integers(0, 256, plen).astype(np.uint8)
        sub = O.tx_packet_freq(pay, mod, cod).astype(np.float64)       # [nsym,48,2]
        ns = sub.shape[0] + extra_sym
        X = np.zeros((ns, 64), np.complex128)
        X[: sub.shape[0], DATA_BINS] = (sub[..., 0] + 1j * sub[..., 1]) / 100.0
        X[: sub.shape[0], PILOT_BINS] = 107.0 * rng.choice([-1.0, 1.0], (sub.shape[0], 4))
        x = np.fft.ifft(X, axis=1) * 64.0
        x = x + rng.normal(0.0, sigma, x.shape) + 1j * rng.normal(0.0, sigma, x.shape)
        t = np.stack([np.rint(x.real), np.rint(x.imag)], -1)
        syms.append(np.clip(t, -32768, 32767).astype(np.int16))
        offs.append(off)
        nsyms.append(ns)
        meta.append((mod, cod, plen + 4))
        off += ns
    return (np.concatenate(syms), np.array(offs, np.int64), np.array(nsyms, np.int32),
            np.array(meta, np.int32))


def pilot_polarity(k):
    """+1 / -1 pilot polarity PilotTrack expects on symbol k of a packet (k = 0: SIGNAL),
    pilotSgn[k == 0 ? 127 : (k-1) % 127] (PilotTrack.blk:70-78, map_ofdm.blk:55-62)."""
    sc = 127 if k == 0 else (k - 1) % 127
    return -1.0 if O.lib().zo_pilot_sign(sc) == -1 else 1.0


def packets_time_eq(plan, seed, sigma=3.0):
    """Packets through a frequency-selective channel for the ChannelEqualization +
    PilotTrack path: per packet a 3-tap channel H and a per-symbol common phase drift plus a
    small phase slope across subcarriers; pilots carry the 802.11a polarity (TX pilots
    +, -, +, + on bins 7, 21, 43, 57 before polarity, map_ofdm.blk:40-49, 86-96).  The
    channel coefficients handed to ChannelEqualization are round(256 / H) (what an ideal
    LTS stage would give at norm_shift 8).  Returns (sym, sym_off, nsym, meta, chan int16
    [n, 64, 2])."""
    rng = np.random.default_rng(seed)
    syms, offs, nsyms, meta, chans = [], [], [], [], []
    off = 0
    b = np.arange(64)
    sb = np.where(b < 32, b, b - 64).astype(np.float64)
    for (mod, cod, plen) in plan:
        pay = rng.integers(0, 256, plen).astype(np.uint8)
        sub = O.tx_packet_freq(pay, mod, cod).astype(np.float64)       # [nsym,48,2]
        ns = sub.shape[0]
        X = np.zeros((ns, 64), np.complex128)
        X[:, DATA_BINS] = (sub[..., 0] + 1j * sub[..., 1]) / 100.0
        pol = np.array([pilot_polarity(k) for k in range(ns)])
        X[:, PILOT_BINS] = 107.0 * pol[:, None] * np.array([1.0, -1.0, 1.0, 1.0])
        h = rng.normal(0, 0.15, 3) + 1j * rng.normal(0, 0.15, 3)
        h[0] += 0.7 * np.exp(2j * np.pi * rng.random())
        H = np.fft.fft(h, 64)
        phi = rng.uniform(-np.pi, np.pi) + rng.uniform(-0.02, 0.02) * np.arange(ns)
        slope = rng.uniform(-2e-4, 2e-4) * np.arange(ns)
        Y = X * H[None, :] * np.exp(1j * (phi[:, None] + slope[:, None] * sb[None, :]))
        x = np.fft.ifft(Y, axis=1) * 64.0
        x = x + rng.normal(0.0, sigma, x.shape) + 1j * rng.normal(0.0, sigma, x.shape)
        t = np.stack([np.rint(x.real), np.rint(x.imag)], -1)
        syms.append(np.clip(t, -32768, 32767).astype(np.int16))
        G = 256.0 / H
        chans.append(np.clip(np.stack([np.rint(G.real), np.rint(G.imag)], -1), -32768, 32767).astype(np.int16))
        offs.append(off)
        nsyms.append(ns)
        meta.append((mod, cod, plen + 4))
        off += ns
    return (np.concatenate(syms), np.array(offs, np.int64), np.array(nsyms, np.int32),
            np.array(meta, np.int32), np.stack(chans))
