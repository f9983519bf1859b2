"""Generates zrx_tables.h — the constant tables of the HIP engine.

Run: python ziria_amd/csrc/gen_tables.py  (the output is committed; tests/test_tables.py
re-derives it and checks it against the golden fixtures).

* Q15 FFT twiddles twFFTLUT{16,64}_{1,2,3}: clamp(round(32768 e^{-j2pi k n/N}), +-32767)
  (reference csrc/sora_ext_lib_fft_coeffs.hpp:53-78, 298-359).
* Soft-demap LUTs m_bpsk_lut, m_qam16_lut2, m_qam64_lut2, m_qam64_lut3
  (reference code/WiFi/const.blk:74-150), stored run-length below as (value, count) runs
  over the u8 index 0..255 and packed one byte per table into a u32 per index.
* Deinterleaver source maps for N_CBPS = 48/96/192/288
  (reference code/WiFi/receiver/decoding/Deinterleave*.blk; 802.11a formula).
"""
import math
import os

RUNS = {
    "bpsk": [(4, 9), (5, 9), (6, 13), (7, 97), (0, 98), (1, 13), (2, 9), (3, 8)],
    "qam16_2": [(7, 56), (6, 3), (5, 3), (4, 2), (3, 2), (2, 2), (1, 3), (0, 115), (1, 3), (2, 2),
                (3, 2), (4, 2), (5, 3), (6, 3), (7, 55)],
    "qam64_2": [(7, 56), (6, 3), (5, 2), (4, 1), (3, 2), (2, 2), (1, 3), (0, 119), (1, 3), (2, 2),
                (3, 2), (4, 1), (5, 2), (6, 3), (7, 55)],
    "qam64_3": [(0, 25), (1, 3), (2, 2), (3, 1), (4, 2), (5, 2), (6, 3), (7, 49), (6, 3), (5, 1), (4, 2), (3, 2), (2, 2), (1, 2), (0, 59), (1, 2), (2, 2), (3, 2), (4, 2), (5, 1), (6, 3), (7, 49), (6, 3), (5, 2), (4, 2), (3, 1), (2, 2), (1, 3), (0, 24)],
}


def lut(name):
    out = []
    for v, c in RUNS[name]:
        out += [v] * c
    assert len(out) == 256, (name, len(out))
    return out


def twiddle(N, k, n):
    ang = -2.0 * math.pi * k * n / N
    r = math.floor(32768.0 * math.cos(ang) + 0.5)
    i = math.floor(32768.0 * math.sin(ang) + 0.5)
    clamp = lambda v: max(-32767, min(32767, v))
    return clamp(r), clamp(i)


def deint_src(ncbps, k):
    nbpsc = ncbps // 48
    s = max(nbpsc // 2, 1)
    i = (ncbps // 16) * (k % 16) + k // 16
    return s * (i // s) + (i + ncbps - (16 * i) // ncbps) % s


def crc_table():
    """Reflected CRC-32 (0x04C11DB7 <-> 0xEDB88320) byte table; equals the bitwise
    update_crc_generic of crc.blk:41-73 (checked by tests against the oracle)."""
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ (0xEDB88320 if c & 1 else 0)
        t.append(c)
    return t


def crc_zero_mats(nk=13):
    """M_k = register map of 2^k zero bytes (column i = image of bit i)."""
    T = crc_table()
    z1 = lambda r: T[r & 0xFF] ^ (r >> 8)
    mats = [[z1(1 << i) for i in range(32)]]
    apply = lambda M, v: __import__("functools").reduce(lambda a, i: a ^ (M[i] if (v >> i) & 1 else 0), range(32), 0)
    for _ in range(1, nk):
        M = mats[-1]
        mats.append([apply(M, M[i]) for i in range(32)])
    return mats


def scrambler_tables():
    """802.11a scrambler x^7+x^4+1 as in scramble.blk:28-44 with state bit k = st[k]:
    t = st[3]^st[0]; shift down; st[6] = t.  seq[p] = state after p steps from state 1;
    phase[s] = p with seq[p] = s (phase[0] = 255: stuck state); kb[p] = keystream byte whose
    bit j is the output of step p+j+1 counted from seq[0]."""
    seq = [1]
    for _ in range(126):
        s = seq[-1]
        t = ((s >> 3) ^ s) & 1
        seq.append((s >> 1) | (t << 6))
    phase = [255] * 128
    for p, s in enumerate(seq):
        phase[s] = p
    kb = []
    for p in range(127):
        b = 0
        for j in range(8):
            b |= ((seq[(p + j + 1) % 127] >> 6) & 1) << j
        kb.append(b)
    return phase, kb


def scrambler_stream(kb):
    """B[n] = kb[(8 n) % 127]: byte q of the keystream of a packet whose scrambler phase is
    ph is B[(16 ph + q) % 127] (8 * 16 = 128 = 1 mod 127), i.e. one cyclic byte sequence.
    Returns B doubled (254 bytes, so B[m + k] needs no wrap for m < 127, k < 127) and the
    little-endian dwords W[n] = B[n] | B[n+1] << 8 | B[n+2] << 16 | B[n+3] << 24 (mod 127)."""
    B = [kb[(8 * n) % 127] for n in range(127)]
    W = [B[n] | (B[(n + 1) % 127] << 8) | (B[(n + 2) % 127] << 16) | (B[(n + 3) % 127] << 24)
         for n in range(127)]
    return B + B, W


def crc_shift_tables(mats):
    """Nibble-sliced register maps of 32 * 2^k zero bytes, k = 0..5: T[k][j][v] = image of
    (v << 4j), so advancing a register r is T[k][0][r&15] ^ ... ^ T[k][7][r>>28]."""
    out = []
    for k in range(5, 11):
        M = mats[k]
        for j in range(8):
            for v in range(16):
                x, r = v << (4 * j), 0
                for i in range(32):
                    if (x >> i) & 1:
                        r ^= M[i]
                out.append(r)
    return out


def crc_shift_n_tables(mats, unit_bytes):
    """Nibble-sliced register maps of n * unit_bytes zero bytes, n = 0..7 (n = 0: identity):
    T[n][j][v] = image of (v << 4j) after those bytes (k_descramble_crc advances a lane's
    register by 32 * (63 - lane) bytes as (63 - lane) & 7 chunks, then (63 - lane) >> 3 x 256)."""
    apply = lambda M, v: __import__("functools").reduce(lambda a, i: a ^ (M[i] if (v >> i) & 1 else 0), range(32), 0)
    out = []
    for n in range(8):
        nbytes = n * unit_bytes
        ks = [k for k in range(len(mats)) if (nbytes >> k) & 1]
        for j in range(8):
            for v in range(16):
                r = v << (4 * j)
                for k in ks:
                    r = apply(mats[k], r)
                out.append(r)
    return out


def crc_ones_shift(n_max=2048):
    """A^n(0xFFFFFFFF), n < n_max: the register an all-ones initial value becomes after n
    zero bytes.  By linearity the reference's CRC (all-ones init, crc.blk:85-118) of n bytes
    is ~(U0(data) ^ A^n(~0)) with U0 the zero-initialised register, so k_descramble_crc runs
    the zero-initialised CRC on the payload as it is and corrects with one table word."""
    T = crc_table()
    out, r = [], 0xFFFFFFFF
    for _ in range(n_max):
        out.append(r)
        r = T[r & 0xFF] ^ (r >> 8)
    return out


def crc_slice4():
    """Slicing-by-4 tables: S[0] = the byte table, S[k][b] = S[k-1][b] after one zero byte."""
    T = crc_table()
    S = [T]
    for _ in range(3):
        S.append([(v >> 8) ^ T[v & 0xFF] for v in S[-1]])
    return S


def pilot_neg_bits():
    """pilotSgn (PilotTrack.blk:70-78) as a 128-bit mask, bit m set = -1.  Entry m is the
    802.11a pilot polarity p_{(m+1) mod 127}, the scrambler output (scramble.blk:28-44) from
    the all-ones state; both reference tables (also allPilotSgn, map_ofdm.blk:30-38) hold
    +1 at entry 52 where the standard has p_53 = -1, kept as in the reference."""
    s, p = [1] * 7, []
    for _ in range(127):
        t = s[3] ^ s[0]
        s = s[1:] + [t]
        p.append(t)
    neg = [p[(m + 1) % 127] for m in range(128)]
    neg[52] = 0
    return [sum(neg[32 * w + b] << b for b in range(32)) for w in range(4)]


def render():
    L = ["// GENERATED by gen_tables.py — do not edit.", "#pragma once", "#include <stdint.h>", ""]
    for N in (16, 32, 64, 128):
        for k in (1, 2, 3):
            vals = [twiddle(N, k, n) for n in range(N // 4)]
            L.append(f"// twFFTLUT{N}_{k} (csrc/sora_ext_lib_fft_coeffs.hpp), (re, im)")
            L.append(f"static constexpr int16_t kTw{N}_{k}[{N // 2}] = {{" +
                     ", ".join(f"{r}, {i}" for r, i in vals) + "};")
    packed = []
    luts = [lut(n) for n in ("bpsk", "qam16_2", "qam64_2", "qam64_3")]
    for i in range(256):
        packed.append(luts[0][i] | (luts[1][i] << 8) | (luts[2][i] << 16) | (luts[3][i] << 24))
    L.append("// byte0 m_bpsk_lut, byte1 m_qam16_lut2, byte2 m_qam64_lut2, byte3 m_qam64_lut3")
    L.append("// (code/WiFi/const.blk:74-150), indexed by the DemapLimit u8 value")
    L.append("static constexpr uint32_t kDemapLut[256] = {" +
             ", ".join(f"0x{v:08x}u" for v in packed) + "};")
    for N in (48, 96, 192, 288):
        L.append(f"// Deinterleave (N_CBPS={N}): out[k] = in[kDeint{N}[k]]")
        L.append(f"static constexpr uint16_t kDeint{N}[{N}] = {{" +
                 ", ".join(str(deint_src(N, k)) for k in range(N)) + "};")
    for N in (48, 96, 192, 288):
        inv = [0] * N
        for k in range(N):
            inv[deint_src(N, k)] = k
        L.append(f"// Interleave (N_CBPS={N}, interleaving.blk): interleaved bit j = coded bit kIntlv{N}[j]")
        L.append(f"static constexpr uint16_t kIntlv{N}[{N}] = {{" + ", ".join(map(str, inv)) + "};")
    L.append("// reflected CRC-32 byte table (crc.blk:41-73, base32 = 0x04C11DB7)")
    L.append("static constexpr uint32_t kCrcTab[256] = {" + ", ".join(f"0x{v:08x}u" for v in crc_table()) + "};")
    L.append("// kCrcZero[k][i]: CRC register image of bit i after 2^k zero bytes")
    L.append("static constexpr uint32_t kCrcZero[13][32] = {" + ", ".join(
        "{" + ", ".join(f"0x{v:08x}u" for v in M) + "}" for M in crc_zero_mats(13)) + "};")
    ph, kb = scrambler_tables()
    L.append("// scrambler (scramble.blk:28-44): phase of a 7-bit state, keystream byte by phase")
    L.append("static constexpr uint8_t kScrPhase[128] = {" + ", ".join(map(str, ph)) + "};")
    L.append("static constexpr uint8_t kScrByte[127] = {" + ", ".join(map(str, kb)) + "};")
    B2, W = scrambler_stream(kb)
    L.append("// keystream byte q of a packet with scrambler phase ph: kScrB2[(16*ph + q) % 127 + ...]")
    L.append("static constexpr uint8_t kScrB2[254] = {" + ", ".join(map(str, B2)) + "};")
    L.append("static constexpr uint32_t kScrW[127] = {" + ", ".join(f"0x{v:08x}u" for v in W) + "};")
    mats = crc_zero_mats(11)
    for name, unit in (("kCrcShiftLo", 32), ("kCrcShiftHi", 256)):
        Tn = crc_shift_n_tables(mats, unit)
        L.append(f"// {name}[n][j*16+v]: CRC register image of (v << 4j) after n * {unit} zero bytes")
        L.append(f"static constexpr uint32_t {name}[8][128] = {{" + ", ".join(
            "{" + ", ".join(f"0x{x:08x}u" for x in Tn[128 * n:128 * n + 128]) + "}" for n in range(8)) + "};")
    T = crc_shift_tables(mats)
    L.append("// kCrcShift[k][j*16+v]: CRC register image of (v << 4j) after 32 * 2^k zero bytes")
    L.append("static constexpr uint32_t kCrcShift[6][128] = {" + ", ".join(
        "{" + ", ".join(f"0x{v:08x}u" for v in T[k * 128:(k + 1) * 128]) + "}" for k in range(6)) + "};")
    S4 = crc_slice4()
    L.append("// kCrcOnes[n]: the all-ones CRC register after n zero bytes (crc_ones_shift)")
    L.append("static constexpr uint32_t kCrcOnes[2048] = {" + ", ".join(f"0x{v:08x}u" for v in crc_ones_shift()) + "};")
    L.append("// slicing-by-4 CRC tables: kCrcS4[k][b] = byte table entry advanced by k zero bytes")
    L.append("static constexpr uint32_t kCrcS4[4][256] = {" + ", ".join(
        "{" + ", ".join(f"0x{v:08x}u" for v in S) + "}" for S in S4) + "};")
    lts = [0, 1, 0, 0, 1, 1, 0, 1, 0, 1, 0, 0, 0, 0, 0, 1, 1, 0, 0, 1, 0, 1, 0, 1, 1, 1, 1, 0, 0, 0, 0, 0,
           0, 0, 0, 0, 0, 0, 1, 1, 0, 0, 1, 1, 0, 1, 0, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1, 0, 1, 0, 1, 1, 1, 1]
    L.append("// lts11a (OFDM/LTS.blk:45-49) as a bit mask: bit b set = LTS bin b is +1")
    L.append(f"static constexpr uint64_t kLts11aBits = 0x{sum(v << b for b, v in enumerate(lts)):016x}ull;")
    st, key = [1, 0, 1, 1, 1, 0, 1], []
    for _ in range(127):
        t = st[3] ^ st[0]
        st = st[1:] + [t]
        key.append(t)
    L.append("// TX scrambler keystream (scramble.blk:28-44, default_scrmbl_st = 1011101): bit m of kTxKey")
    L.append("static constexpr uint32_t kTxKey[4] = {" + ", ".join(
        f"0x{sum(key[32 * w + b] << b for b in range(32) if 32 * w + b < 127):08x}u" for w in range(4)) + "};")
    L.append("// pilotSgn (PilotTrack.blk:70-78): bit m of kPilotNeg = entry m is -1")
    L.append("static constexpr uint32_t kPilotNeg[4] = {" + ", ".join(f"0x{v:08x}u" for v in pilot_neg_bits()) + "};")
    return "\n".join(L) + "\n"


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "zrx_tables.h"), "w") as f:
        f.write(render())
