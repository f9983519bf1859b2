"""Engine constant tables and the bench workload generator, checked on the CPU."""
import os
import re
import zlib

import numpy as np

from ziria_amd import txgen

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_arrays():
    txt = open(os.path.join(ROOT, "ziria_amd", "csrc", "zrx_tables.h")).read()
    out = {}
    for m in re.finditer(r"static constexpr \w+ (\w+)\[(\d+)\](?:\[(\d+)\])? = \{(.*?)\};", txt, re.S):
        vals = [int(v.strip().rstrip("u"), 0) for v in m.group(4).replace("{", "").replace("}", "").split(",")]
        out[m.group(1)] = np.array(vals, np.int64)
    return out


def test_generated_header_is_current():
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_tables", os.path.join(ROOT, "ziria_amd", "csrc", "gen_tables.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    assert open(os.path.join(ROOT, "ziria_amd", "csrc", "zrx_tables.h")).read() == g.render()


def test_demap_lut_matches_reference(golden):
    t = golden["ref_tables"]
    lut = _header_arrays()["kDemapLut"]
    for byte, n in enumerate(("m_bpsk_lut", "m_qam16_lut2", "m_qam64_lut2", "m_qam64_lut3")):
        assert (((lut >> (8 * byte)) & 0xFF) == t[n]).all(), n


def test_deinterleave_matches_reference(golden):
    a = _header_arrays()
    for mod, n in enumerate((48, 96, 192, 288)):
        assert (a[f"kDeint{n}"] == golden["ref_tables"][f"deint_{mod}"]).all()


def test_twiddles_match_oracle(oracle):
    a = _header_arrays()
    for N in (16, 64):
        for k in (1, 2, 3):
            tw = a[f"kTw{N}_{k}"].reshape(-1, 2)
            for n in range(N // 4):
                assert tuple(tw[n]) == oracle.twiddle(N, k, n)


def test_crc_tables():
    a = _header_arrays()
    tab = a["kCrcTab"]
    data = bytes(range(200))
    reg = 0xFFFFFFFF
    for b in data:
        reg = int(tab[(reg ^ b) & 0xFF]) ^ (reg >> 8)
    assert reg ^ 0xFFFFFFFF == zlib.crc32(data)
    Z = a["kCrcZero"].reshape(13, 32)
    def apply(M, v):
        r = 0
        for i in range(32):
            if (v >> i) & 1:
                r ^= int(M[i])
        return r
    v = 0x12345678
    for k in range(5):
        w = v
        for _ in range(1 << k):
            w = int(tab[w & 0xFF]) ^ (w >> 8)
        assert apply(Z[k], v) == w


def test_crc_ones_identity():
    """k_descramble_crc's form of the reference CRC (all-ones init, crc.blk:85-118 = zlib):
    the zero-initialised register of the payload XOR kCrcOnes[n], complemented, for payloads
    of every length class the kernel sees (its < 4-byte path aside)."""
    a = _header_arrays()
    tab, ones = a["kCrcTab"], a["kCrcOnes"]
    rng = np.random.default_rng(5)
    for n in (4, 5, 31, 32, 33, 255, 1500, 2043, 2044):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        reg = 0
        for b in data:
            reg = int(tab[(reg ^ b) & 0xFF]) ^ (reg >> 8)
        assert (~(reg ^ int(ones[n]))) & 0xFFFFFFFF == zlib.crc32(data), n


def test_scrambler_tables():
    a = _header_arrays()
    phase, kb = a["kScrPhase"], a["kScrByte"]
    ks = txgen._scrambler_keystream(200)           # from state 1011101
    st = sum(((0b1011101 >> (6 - k)) & 1) << k for k in range(7))
    p = int(phase[st])
    for q in range(20):
        byte = int(kb[(p + 8 * q) % 127])
        assert byte == int(np.packbits(ks[8 * q:8 * q + 8], bitorder="little")[0])


def test_txgen_matches_oracle_transmitter(oracle):
    rng = np.random.default_rng(3)
    for mod, cod in txgen.MCS8:
        for L in (60, 101, 1500):
            pay = rng.integers(0, 256, (2, L), dtype=np.uint8)
            f = txgen.packets_freq(pay, mod, cod).numpy()
            for i in range(2):
                assert (oracle.tx_packet_freq(pay[i], mod, cod) == f[i]).all(), (mod, cod, L)


def test_txgen_batch_decodes_in_oracle(oracle):
    b = txgen.make_batch(16, seed=21)
    pay, res = oracle.rx_batch_time(b["sym"].numpy(), b["sym_off"].numpy(), b["nsym"].numpy(), nthreads=4)
    assert all(r["crc_ok"] == 1 for r in res)
    assert (pay[:, :1500] == b["payload"]).all()


def test_txgen_mixed_decodes_in_oracle(oracle):
    m = txgen.make_mixed(24, max_len=900, seed=8)
    pay, res = oracle.rx_batch_time(m["sym"].numpy(), m["sym_off"].numpy(), m["nsym"].numpy(), nthreads=4)
    for i, r in enumerate(res):
        assert r["crc_ok"] == 1 and (r["modulation"], r["coding"], r["len"]) == tuple(m["meta"][i])
        assert (pay[i, :r["len"] - 4] == m["payload"][i]).all()


def test_txgen_mixed_fast_decodes_in_oracle(oracle):
    """The vectorized config-5 generator: every packet distinct, all 8 MCS, header lengths up
    to 4095 (those above 2048 are header errors the receiver must flag)."""
    m = txgen.make_mixed_fast(48, min_len=64, max_len=2600, sigma=3.0, seed=9, chunk=5)
    pay, res = oracle.rx_batch_time(m["sym"].numpy(), m["sym_off"].numpy(), m["nsym"].numpy(), nthreads=4)
    assert len({p.tobytes() for p in m["payload"]}) == 48
    assert len({int(x) for x in m["meta"][:, 0] * 4 + m["meta"][:, 1]}) >= 6
    for i, r in enumerate(res):
        if m["meta"][i, 2] > 2048:
            assert r["crc_ok"] != 1
            continue
        assert r["crc_ok"] == 1 and (r["modulation"], r["coding"], r["len"]) == tuple(m["meta"][i])
        assert (pay[i, :r["len"] - 4] == m["payload"][i]).all()
