"""Synthetic 802.11a packet workloads (BASELINE configs 2, 3, 5), vectorized in torch so
that a 16k-packet batch is generated in seconds (on the GPU when one is present).

This is a workload generator, not part of the decode path.  It restates the transmitter
(code/WiFi/transmitter/transmitter.blk:56-101: crc + SERVICE + pad, scrambler 1011101,
encode12/23/34, interleave, modulate) and the channel of SURVEY.md Appendix E:
x = IDFT(X / 100) * 64 + N(0, sigma^2) per component, rounded to int16.
tests/test_tables_txgen.py checks it against the oracle's transmitter restatement.
"""
import zlib

import numpy as np
import torch

NCBPS = {0: 48, 1: 96, 2: 192, 3: 288}
UNIT = {0: 10720, 1: 7581, 2: 3390, 3: 1654}          # const.blk:27-30 (int16 of the quotient)
DATA_BINS = (list(range(38, 43)) + list(range(44, 57)) + list(range(58, 64)) + list(range(1, 7)) +
             list(range(8, 21)) + list(range(22, 27)))       # GetData.blk:24-35
PILOT_BINS = [7, 21, 43, 57]
RATE_NIBBLE = {(0, 0): 0xB, (0, 2): 0xF, (1, 0): 0xA, (1, 2): 0xE, (2, 0): 0x9, (2, 2): 0xD,
               (3, 1): 0x8, (3, 2): 0xC}


def ndbps(mod, coding):
    nc = NCBPS[mod]
    return nc // 2 if coding == 0 else (nc * 2 // 3 if coding == 1 else nc * 3 // 4)


def n_data_symbols(mod, coding, payload_len):
    """Data OFDM symbols for a payload of payload_len bytes (+4 CRC)."""
    nd = ndbps(mod, coding)
    return (16 + 8 * payload_len + 32 + 6 + nd - 1) // nd


def interleave_perm(mod):
    """p(k) of the 802.11a interleaver (interleaving.blk:38-58); TX: out[p(k)] = in[k]."""
    N = NCBPS[mod]
    s = max(N // 48 // 2, 1)
    k = np.arange(N)
    i = (N // 16) * (k % 16) + k // 16
    return s * (i // s) + (i + N - (16 * i) // N) % s


def _scrambler_keystream(n, state=None):
    """Keystream bits of the x^7+x^4+1 scrambler (scramble.blk:28-44) from a 7-bit initial
    state (bit k = st[k]); default default_scrmbl_st = 1011101 (scramble.blk:22)."""
    st = [1, 0, 1, 1, 1, 0, 1] if state is None else [(int(state) >> k) & 1 for k in range(7)]
    out = np.zeros(n, np.uint8)
    for k in range(n):
        t = st[3] ^ st[0]
        st = st[1:] + [t]
        out[k] = t
    return out


def _encode(u, coding):
    """u: uint8 [n, L] bits -> punctured coded bits (encoding.blk:24-109)."""
    n, L = u.shape
    z = torch.zeros((n, 6), dtype=u.dtype, device=u.device)
    p = torch.cat([z, u], 1)
    d = lambda k: p[:, 6 - k: 6 - k + L]             # u[n-k]
    A = d(0) ^ d(2) ^ d(3) ^ d(5) ^ d(6)
    B = d(0) ^ d(1) ^ d(2) ^ d(3) ^ d(6)
    if coding == 0:
        return torch.stack([A, B], 2).reshape(n, 2 * L)
    if coding == 2:                                  # A0 B0 A1 B2 per 3 input bits
        A3, B3 = A.reshape(n, L // 3, 3), B.reshape(n, L // 3, 3)
        return torch.stack([A3[..., 0], B3[..., 0], A3[..., 1], B3[..., 2]], 2).reshape(n, -1)
    A2, B2 = A.reshape(n, L // 2, 2), B.reshape(n, L // 2, 2)   # 2/3: A0 B0 A1
    return torch.stack([A2[..., 0], B2[..., 0], A2[..., 1]], 2).reshape(n, -1)


def _map(bits, mod):
    """bits uint8 [..., nbpsc] -> (re, im) levels in units (modulating.blk)."""
    b = bits.to(torch.int64)
    if mod == 0:
        return (2 * b[..., 0] - 1), torch.zeros_like(b[..., 0])
    if mod == 1:
        return 2 * b[..., 0] - 1, 2 * b[..., 1] - 1
    if mod == 2:
        g = torch.tensor([-3, -1, 3, 1], device=bits.device)
        return g[2 * b[..., 0] + b[..., 1]], g[2 * b[..., 2] + b[..., 3]]
    g = torch.tensor([-7, -5, -1, -3, 7, 5, 1, 3], device=bits.device)
    return g[4 * b[..., 0] + 2 * b[..., 1] + b[..., 2]], g[4 * b[..., 3] + 2 * b[..., 4] + b[..., 5]]


def _signal_levels(mod, coding, length, device):
    h = np.zeros(24, np.uint8)
    code = RATE_NIBBLE[(mod, coding)]
    h[0:4] = [(code >> k) & 1 for k in range(4)]
    h[5:17] = [(length >> k) & 1 for k in range(12)]
    h[17] ^= h.sum() & 1
    coded = _encode(torch.from_numpy(h[None]).to(device), 0)[0]
    il = torch.empty_like(coded)
    il[torch.from_numpy(interleave_perm(0)).to(device)] = coded
    re, _ = _map(il[:, None], 0)
    return re * UNIT[0]


def packets_freq(payloads, mod, coding, device="cpu", scrambler=None):
    """Frequency-domain symbols (GetData order, TX units) for equal-length payloads.
    payloads: uint8 numpy [n, L]; scrambler: None (the default state for every packet) or
    one 7-bit initial scrambler state per packet.  Returns int64 torch [n, 1 + nsym, 48, 2]."""
    n, L = payloads.shape
    nd, nc = ndbps(mod, coding), NCBPS[mod]
    nsym = n_data_symbols(mod, coding, L)
    nbits = nsym * nd
    bits = np.zeros((n, nbits), np.uint8)
    bits[:, 16:16 + 8 * L] = np.unpackbits(payloads, axis=1, bitorder="little")
    crc = np.array([zlib.crc32(p.tobytes()) for p in payloads], np.uint32)
    bits[:, 16 + 8 * L:16 + 8 * L + 32] = ((crc[:, None] >> np.arange(32, dtype=np.uint32)) & 1).astype(np.uint8)
    if scrambler is None:
        bits ^= _scrambler_keystream(nbits)[None]
    else:
        ks = {int(v): _scrambler_keystream(nbits, v) for v in np.unique(scrambler)}
        bits ^= np.stack([ks[int(v)] for v in scrambler])
    u = torch.from_numpy(bits).to(device)
    coded = _encode(u, coding).reshape(n, nsym, nc)
    perm = torch.from_numpy(interleave_perm(mod)).to(device)
    il = torch.empty_like(coded)
    il[:, :, perm] = coded
    re, im = _map(il.reshape(n, nsym, 48, nc // 48), mod)
    out = torch.zeros((n, 1 + nsym, 48, 2), dtype=torch.int64, device=device)
    out[:, 1:, :, 0] = re * UNIT[mod]
    out[:, 1:, :, 1] = im * UNIT[mod]
    out[:, 0, :, 0] = _signal_levels(mod, coding, L + 4, device)
    return out


def pilot_polarity(S):
    """+1/-1 pilot polarity of symbols 0..S-1 of a packet (0 = SIGNAL) as PilotTrack reads
    it: pilotSgn[k == 0 ? 127 : (k-1) % 127] (PilotTrack.blk:70-78, map_ofdm.blk:55-62), the
    802.11a sequence with the reference tables' +1 at entry 52."""
    s, p = [1] * 7, []
    for _ in range(127):
        t = s[3] ^ s[0]
        s = s[1:] + [t]
        p.append(t)
    sgn = [-1.0 if p[(m + 1) % 127] else 1.0 for m in range(128)]
    sgn[52] = 1.0
    return np.array([sgn[127 if k == 0 else (k - 1) % 127] for k in range(S)], np.float32)


def to_time(freq, sigma, gen, atten=100.0, channel=False):
    """freq int64 [n, S, 48, 2] -> time-domain int16 [n, S, 64, 2] (Appendix E channel).
    channel=True: pilots with the 802.11a polarity (+,-,+,+ on bins 7,21,43,57,
    map_ofdm.blk:40-49), a 3-tap channel H per packet, a common phase drift per symbol and a
    small phase slope across subcarriers; returns (sym, chan) with chan int16 [n,64,2] =
    round(256 / H), the coefficients ChannelEqualization (norm_shift 8) takes."""
    n, S = freq.shape[:2]
    dev = freq.device
    X = torch.zeros((n, S, 64), dtype=torch.complex64, device=dev)
    bins = torch.tensor(DATA_BINS, device=dev)
    X[:, :, bins] = torch.complex(freq[..., 0].float(), freq[..., 1].float()) / atten
    pbins = torch.tensor(PILOT_BINS, device=dev)
    if channel:
        pol = torch.from_numpy(pilot_polarity(S)).to(dev)
        pil = 107.0 * pol[None, :, None] * torch.tensor([1.0, -1.0, 1.0, 1.0], device=dev)
        X[:, :, pbins] = torch.complex(pil.expand(n, S, 4).contiguous(), torch.zeros((n, S, 4), device=dev))
        h = torch.complex(torch.randn((n, 3), generator=gen, device=dev), torch.randn((n, 3), generator=gen, device=dev)) * 0.1
        ph0 = torch.rand((n,), generator=gen, device=dev) * 2 * np.pi
        h[:, 0] += 0.7 * torch.exp(torch.complex(torch.zeros_like(ph0), ph0))
        H = torch.fft.fft(h, n=64, dim=-1)                                   # [n, 64]
        k = torch.arange(S, device=dev, dtype=torch.float32)
        drift = (torch.rand((n, 1), generator=gen, device=dev) * 2 - 1) * 0.02
        slope = (torch.rand((n, 1), generator=gen, device=dev) * 2 - 1) * 2e-4
        b = torch.arange(64, device=dev)
        sb = torch.where(b < 32, b, b - 64).float()
        ang = (drift * k)[:, :, None] + (slope * k)[:, :, None] * sb[None, None, :]
        X = X * H[:, None, :] * torch.exp(torch.complex(torch.zeros_like(ang), ang))
        G = 256.0 / H
        chan = torch.clamp(torch.round(torch.stack([G.real, G.imag], -1)), -32768, 32767).to(torch.int16)
    else:
        pil = (torch.randint(0, 2, (n, S, 4), generator=gen, device=dev) * 2 - 1).float() * 107.0
        X[:, :, pbins] = torch.complex(pil, torch.zeros_like(pil))
    x = torch.fft.ifft(X, dim=-1) * 64.0
    t = torch.stack([x.real, x.imag], -1)
    if sigma > 0:
        t = t + sigma * torch.randn(t.shape, generator=gen, device=dev)
    t = torch.clamp(torch.round(t), -32768, 32767).to(torch.int16)
    return (t, chan) if channel else t


def make_batch(n, mod=3, coding=2, payload_len=1500, sigma=4.0, seed=0x5EED, device="cpu", chunk=2048,
               channel=False, scrambler=None):
    """BASELINE config 3 shape by default: n packets of payload_len bytes at (mod, coding).
    Returns dict(sym int16 [n*S,64,2], sym_off int64 [n], nsym int32 [n], payload uint8
    [n, L], max_nsym); channel=True adds the channel of to_time and chan int16 [n,64,2];
    scrambler: per-packet initial scrambler states (packets_freq), default the reference's."""
    rng = np.random.default_rng(seed)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    payloads = rng.integers(0, 256, (n, payload_len), dtype=np.uint8)
    syms, chans = [], []
    for a in range(0, n, chunk):
        f = packets_freq(payloads[a:a + chunk], mod, coding, device,
                         scrambler=None if scrambler is None else np.asarray(scrambler)[a:a + chunk])
        t = to_time(f, sigma, gen, channel=channel)
        if channel:
            t, c = t
            chans.append(c)
        syms.append(t.reshape(-1, 64, 2))
    S = 1 + n_data_symbols(mod, coding, payload_len)
    sym = torch.cat(syms, 0)
    d = dict(sym=sym, sym_off=torch.arange(n, dtype=torch.int64, device=device) * S,
             nsym=torch.full((n,), S, dtype=torch.int32, device=device), payload=payloads,
             max_nsym=S, mod=mod, coding=coding, payload_len=payload_len)
    if channel:
        d["chan"] = torch.cat(chans, 0).contiguous()
    return d


MCS8 = [(0, 0), (0, 2), (1, 0), (1, 2), (2, 0), (2, 2), (3, 1), (3, 2)]


def _signal_levels_batch(mod, coding, lengths, device):
    """_signal_levels for many packets of one MCS: int64 [n, 48] BPSK levels."""
    n = len(lengths)
    h = np.zeros((n, 24), np.uint8)
    code = RATE_NIBBLE[(mod, coding)]
    h[:, 0:4] = [(code >> k) & 1 for k in range(4)]
    L = np.asarray(lengths, np.int64)
    h[:, 5:17] = (L[:, None] >> np.arange(12)) & 1
    h[:, 17] ^= (h.sum(1) & 1).astype(np.uint8)
    coded = _encode(torch.from_numpy(h).to(device), 0)
    il = torch.empty_like(coded)
    il[:, torch.from_numpy(interleave_perm(0)).to(device)] = coded
    re, _ = _map(il[..., None], 0)
    return re * UNIT[0]


def make_mixed_fast(n, min_len=64, max_len=4095, sigma=4.0, seed=0x3C5, device="cpu", chunk=1024):
    """BASELINE config 5 with n distinct packets, vectorized per MCS: the same transmitter and
    channel as make_mixed (MCS uniform over the 8 rates, PSDU length uniform in [min_len,
    max_len]), packets of one MCS built together on zero-padded bit arrays (the encoder is
    causal, so a packet's own symbols do not depend on the padding).  Packet i's payload,
    MCS and length come from one seeded generator in packet order; its noise from the
    chunk it is built in."""
    rng = np.random.default_rng(seed)
    mcs = rng.integers(0, 8, n)
    lens = rng.integers(min_len, max_len + 1, n)
    pays = [rng.integers(0, 256, int(lens[i]) - 4, dtype=np.uint8) for i in range(n)]
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    sym_of = [None] * n
    for m in range(8):
        mod, cod = MCS8[m]
        idx = np.nonzero(mcs == m)[0]
        nd = ndbps(mod, cod)
        for a in range(0, idx.size, chunk):
            ids = idx[a:a + chunk]
            Ls = lens[ids] - 4
            nsyms = np.array([n_data_symbols(mod, cod, int(L)) for L in Ls])
            S = int(nsyms.max())
            nbits = S * nd
            maxL = int(Ls.max())
            byt = np.zeros((ids.size, maxL), np.uint8)
            for r, i in enumerate(ids):
                byt[r, :Ls[r]] = pays[i]
            bits = np.zeros((ids.size, nbits), np.uint8)
            bits[:, 16:16 + 8 * maxL] = np.unpackbits(byt, axis=1, bitorder="little")
            crc = np.array([zlib.crc32(pays[i].tobytes()) for i in ids], np.uint32)
            cpos = 16 + 8 * Ls[:, None] + np.arange(32)[None, :]
            bits[np.arange(ids.size)[:, None], cpos] = ((crc[:, None] >> np.arange(32, dtype=np.uint32)) & 1).astype(np.uint8)
            bits ^= _scrambler_keystream(nbits)[None]
            u = torch.from_numpy(bits).to(device)
            nc = NCBPS[mod]
            coded = _encode(u, cod).reshape(ids.size, S, nc)
            perm = torch.from_numpy(interleave_perm(mod)).to(device)
            il = torch.empty_like(coded)
            il[:, :, perm] = coded
            re, im = _map(il.reshape(ids.size, S, 48, nc // 48), mod)
            f = torch.zeros((ids.size, 1 + S, 48, 2), dtype=torch.int64, device=device)
            f[:, 1:, :, 0] = re * UNIT[mod]
            f[:, 1:, :, 1] = im * UNIT[mod]
            f[:, 0, :, 0] = _signal_levels_batch(mod, cod, lens[ids], device)
            t = to_time(f, sigma, gen)
            for r, i in enumerate(ids):
                sym_of[i] = t[r, :1 + nsyms[r]]
    nsym = [int(x.shape[0]) for x in sym_of]
    off = np.concatenate([[0], np.cumsum(nsym)[:-1]]).astype(np.int64)
    return dict(sym=torch.cat(sym_of, 0).reshape(-1, 64, 2).contiguous(),
                sym_off=torch.from_numpy(off).to(device), nsym=torch.tensor(nsym, dtype=torch.int32, device=device),
                payload=pays, meta=np.stack([np.array([MCS8[int(m)][0] for m in mcs]), np.array([MCS8[int(m)][1] for m in mcs]),
                                             lens], 1).astype(np.int32), max_nsym=int(max(nsym)))


def make_mixed(n, min_len=64, max_len=4095, sigma=4.0, seed=0x3C5, device="cpu", unique=None):
    """BASELINE config 5: MCS uniform over the 8 rates, PSDU length (the PLCP LENGTH field,
    payload + 4 CRC bytes) uniform in [min_len, max_len].  Lengths > 2048 are header errors
    under the reference parser (parsePLCPHeader.blk:171-174) and decode to no payload.
    unique < n: generate `unique` packets (one TX per packet is slow) and tile them."""
    if unique is not None and unique < n:
        m = make_mixed(unique, min_len, max_len, sigma, seed, device)
        reps = (n + unique - 1) // unique
        S = m["sym"].shape[0]
        idx = torch.arange(n, device=device) % unique
        offs = m["sym_off"][idx] + (torch.arange(n, device=device) // unique) * S
        return dict(sym=m["sym"].repeat(reps, 1, 1), sym_off=offs, nsym=m["nsym"][idx],
                    payload=[m["payload"][i % unique] for i in range(n)],
                    meta=m["meta"][np.arange(n) % unique], max_nsym=m["max_nsym"])
    rng = np.random.default_rng(seed)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    mcs = rng.integers(0, 8, n)
    lens = rng.integers(min_len, max_len + 1, n)
    syms, offs, nsyms, pays, meta = [], [], [], [], []
    off = 0
    for i in range(n):
        mod, cod = MCS8[int(mcs[i])]
        L = int(lens[i]) - 4
        pay = rng.integers(0, 256, (1, L), dtype=np.uint8)
        f = packets_freq(pay, mod, cod, device)
        t = to_time(f, sigma, gen).reshape(-1, 64, 2)
        syms.append(t)
        offs.append(off)
        nsyms.append(t.shape[0])
        off += t.shape[0]
        pays.append(pay[0])
        meta.append((mod, cod, L + 4))
    return dict(sym=torch.cat(syms, 0), sym_off=torch.tensor(offs, dtype=torch.int64, device=device),
                nsym=torch.tensor(nsyms, dtype=torch.int32, device=device), payload=pays,
                meta=np.array(meta, np.int32), max_nsym=int(max(nsyms)))


def _chunk_seeds(seed, c):
    return np.random.default_rng([seed, c]), (seed * 1000003 + 7919 * c) & 0x7FFFFFFFFFFF


def payloads_range(lo, hi, payload_len=1500, seed=0x5EED, chunk=2048):
    """Payloads of global packets [lo, hi) of make_batch_range (numpy uint8 [hi-lo, L])."""
    out = []
    for c in range(lo // chunk, (hi + chunk - 1) // chunk):
        rng, _ = _chunk_seeds(seed, c)
        p = rng.integers(0, 256, (chunk, payload_len), dtype=np.uint8)
        a, b = max(lo, c * chunk) - c * chunk, min(hi, (c + 1) * chunk) - c * chunk
        out.append(p[a:b])
    return np.concatenate(out, 0) if out else np.zeros((0, payload_len), np.uint8)


def make_batch_range(lo, hi, mod=3, coding=2, payload_len=1500, sigma=4.0, seed=0x5EED, device="cpu", chunk=2048,
                     channel=False):
    """Global packets [lo, hi) of a batch whose packet i depends only on (seed, i): chunk c
    of `chunk` packets draws its payloads and noise from generators seeded by (seed, c), so
    a rank that builds its contiguous shard gets exactly the packets a single GPU decoding
    the whole batch would (BASELINE config 4: same per-packet outputs).  Same dict as
    make_batch, for the hi-lo packets of the range."""
    S = 1 + n_data_symbols(mod, coding, payload_len)
    syms, chans, pays = [], [], []
    for c in range(lo // chunk, (hi + chunk - 1) // chunk):
        rng, tseed = _chunk_seeds(seed, c)
        p = rng.integers(0, 256, (chunk, payload_len), dtype=np.uint8)
        a, b = max(lo, c * chunk) - c * chunk, min(hi, (c + 1) * chunk) - c * chunk
        gen = torch.Generator(device=device)
        gen.manual_seed(tseed)
        f = packets_freq(p, mod, coding, device)
        t = to_time(f, sigma, gen, channel=channel)
        if channel:
            t, ch = t
            chans.append(ch[a:b])
        syms.append(t[a:b].reshape(-1, 64, 2))
        pays.append(p[a:b])
    n = hi - lo
    d = dict(sym=torch.cat(syms, 0) if syms else torch.zeros((0, 64, 2), dtype=torch.int16, device=device),
             sym_off=torch.arange(n, dtype=torch.int64, device=device) * S,
             nsym=torch.full((n,), S, dtype=torch.int32, device=device),
             payload=np.concatenate(pays, 0) if pays else np.zeros((0, payload_len), np.uint8),
             max_nsym=S, mod=mod, coding=coding, payload_len=payload_len)
    if channel:
        d["chan"] = torch.cat(chans, 0).contiguous()
    return d
