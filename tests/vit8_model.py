"""Executable model of the 8-lane Viterbi row layout (test infrastructure, like vit3_model).

One packet = 8 lanes x 4 dwords x 2 16-bit halves = 64 trellis positions, so a wave holds
8 rows (k_viterbi3 with kLanes = 8).  Position bits 0..2 live inside the lane (half, dword
bits 0 and 1), bits 3..5 are lane bits mapped to lane xor 1, 2, 7: DPP quad_perm, quad_perm
and row_half_mirror inside each 8-lane group.  The column is vit3_model's shift-free step5
(labels rotate: position p holds state rotl6(p, t mod 6); partner bit 5 - t mod 6), with the
round-4 half format: [bit 15: 0][H >> 1 in bits 14..8][the cycle's decisions in bits 7..0, the
column with cycle phase KPH writing its marker at bit KPH], branch metrics halved (BM / 2 =
v ^ (e ? 7 : 0)) so P's bytes are 3-bit soft values, and no carry guard: a half's sum
(H >> 1) + BM / 2 < 256 never leaves its 16 bits, and a wrap of the reference's u8 metric
shows as bit 15, which the guarded column clears after each add (zrx_viterbi3.hpp "Guard-free
columns").  A snapshot byte is bits 7..0 as they are.  What the 8-lane layout changes is
which partner is a DPP move (phases 0..2), a dword swap (phases 3, 4: dword d ^ 2, d ^ 1) or
the half swap (phase 5), and which dwords share a branch-metric word:
  a position bit flips state bit (b + ph) % 6, and flipping state bit 3 changes neither
  expected bit nor the marker, bit 5 only the marker, two bits that each flip A and B
  (bits 1, 2) nothing — see bx_source().
Reference semantics: csrc/sora_ext_viterbi.cpp:66-153 over csrc/viterbicore.hpp:105-239.
"""
import numpy as np

from tests import vit3_model as V3

RING = V3.RING
NL, ND = 8, 4
XOR_OF_BIT = {3: 1, 4: 2, 5: 7}   # position bit -> lane xor (quad_perm / quad_perm / row_half_mirror)


def lane_of(p):
    l = 0
    for b, x in XOR_OF_BIT.items():
        if (p >> b) & 1:
            l ^= x
    return l


def pos_of(lane, d, h):
    l0, l1, l2 = lane & 1, (lane >> 1) & 1, (lane >> 2) & 1
    b5 = l2
    b3, b4 = l0 ^ b5, l1 ^ b5
    return h | (d << 1) | (b3 << 3) | (b4 << 4) | (b5 << 5)


POS = np.array([[[pos_of(l, d, h) for h in range(2)] for d in range(ND)] for l in range(NL)])
assert sorted(POS.ravel().tolist()) == list(range(64))
assert all(lane_of(pos_of(l, d, h)) == l for l in range(NL) for d in range(ND) for h in range(2))


def expected(j):
    """(A, B, marker) of state j (encoding.blk:92-109; marker = branch index j >> 5)."""
    return ((j >> 1) ^ (j >> 2) ^ (j >> 4)) & 1, (j ^ (j >> 1) ^ (j >> 2)) & 1, (j >> 5) & 1


def sel_word(ph, l, d):
    """v_perm selector of (phase, lane, dword): per half [P byte 2A + B][marker byte or 0]."""
    w = 0
    for h in range(2):
        j = V3.rotl6(int(POS[l, d, h]), ph)
        A, B, bm = expected(j)
        w |= (4 if bm else 12) << (16 * h)
        w |= (2 * A + B) << (16 * h + 8)
    return w


SEL = np.array([[[sel_word(ph, l, d) for d in range(ND)] for l in range(NL)] for ph in range(6)], np.uint32)


def bx_source(ph, d):
    """How column phase ph gets dword d's branch-metric word: ('perm',) its own v_perm,
    ('same', e) dword e's word, ('mk', e) dword e's word with the marker bits flipped.
    Derived from which state bits dword bits 0/1 flip at this phase."""
    flips = [(1 + ph) % 6 if d & 1 else None, (2 + ph) % 6 if d & 2 else None]
    flips = [b for b in flips if b is not None]
    a_flip = sum(1 for b in flips if b in (1, 2, 4)) & 1
    b_flip = sum(1 for b in flips if b in (0, 1, 2)) & 1
    m_flip = sum(1 for b in flips if b == 5) & 1
    if d == 0:
        return ("perm",)
    if a_flip == 0 and b_flip == 0:
        return ("mk", 0) if m_flip else ("same", 0)
    # another dword with the same (A, B) flips, if any, lower first
    def flips_of(e):
        fe = [(1 + ph) % 6 if e & 1 else None, (2 + ph) % 6 if e & 2 else None]
        fe = [b for b in fe if b is not None]
        return (sum(1 for b in fe if b in (1, 2, 4)) & 1, sum(1 for b in fe if b in (0, 1, 2)) & 1,
                sum(1 for b in fe if b == 5) & 1)
    for e in range(1, d):
        ae, be, me = flips_of(e)
        if (ae, be) == (a_flip, b_flip):
            return ("mk", e) if me != m_flip else ("same", e)
    # both expected bits flipped against dword e: complementary branch metrics, BX and BY swap
    # roles (zrx_viterbi3.hpp bx_src), the markers flipped unless the marker bit flips too
    for e in range(d):
        ae, be, me = flips_of(e)
        if (ae ^ a_flip, be ^ b_flip) == (1, 1):
            return ("comp", e, me != m_flip)
    return ("perm",)


def partner(T, ph):
    """T [NL, ND] -> the partner's word for every (lane, dword) at phase ph (the half swap of
    phase 5 is applied by the caller's op_sel add)."""
    bit = 5 - ph
    if bit >= 3:
        return T[np.arange(NL) ^ XOR_OF_BIT[bit]]
    if bit == 2:
        return T[:, np.arange(ND) ^ 2]
    if bit == 1:
        return T[:, np.arange(ND) ^ 1]
    return None


class Packet(V3.Packet):
    def __init__(self, frame_len, code_rate):
        self.fl, self.cr = frame_len, code_rate
        st = np.where(POS == 0, 0, 48 >> 1).astype(np.uint32)            # H >> 1 of ALL_INIT0
        self.M = ((st[..., 1] << 24) | (st[..., 0] << 8)).astype(np.uint32)   # [8, 4]
        self.ring = np.zeros((RING, 64), np.uint8)
        self.tr = 0
        self.ob = 0
        self.end = 8 * frame_len + 6
        self.out = []
        self.done = False
        self.v5 = True
        self.guard = True         # False: the guard-free column (zrx_viterbi3.hpp "Guard-free columns")
        self.carries = 0          # halves whose sum set bit 15 (a metric wrap; guard-free: must stay 0)

    def step5(self, kind, a, b):
        ph = self.tr % 6
        c = self.tr + 1
        k = (c + 1) % 8
        T = (self.M & 0x7F007F00).astype(np.uint32) if k == 0 else self.M.copy()
        mk = 1 << k
        P = (V3.p_word(kind, a, b) >> 1) & 0x7F7F7F7F           # BM / 2 per byte
        BX = np.zeros((NL, ND), np.uint32)
        BY = np.zeros((NL, ND), np.uint32)
        mbits = mk * 0x00010001
        K = 14 if kind == V3.FULL else 7
        C = ((K << 8) | mk) * 0x00010001
        sub = lambda x: ((C - x.astype(np.int64)) & 0xFFFFFFFF).astype(np.uint32)
        for d in range(ND):
            src = bx_source(ph, d)
            if src[0] == "comp":
                fl = 0 if src[2] else mbits
                BX[:, d], BY[:, d] = BY[:, src[1]] ^ fl, BX[:, src[1]] ^ fl
                # (the complement identity the kernel relies on, checked on every column)
                assert (BY[:, d] == sub(BX[:, d])).all()
                if ph == 5 and not src[2]:
                    # at the half-partner phase a word's halves hold one branch metric and the
                    # two markers: flipping the markers swaps the halves (column_acs op_sel form)
                    e = src[1]
                    assert (BX[:, d] == V3.swap_halves(BY[:, e])).all()
                    assert (BY[:, d] == V3.swap_halves(BX[:, e])).all()
                continue
            if src[0] == "perm":
                BX[:, d] = V3.perm(mk * 0x01010101, P, SEL[ph, :, d])
            elif src[0] == "same":
                BX[:, d] = BX[:, src[1]]
            else:
                BX[:, d] = BX[:, src[1]] ^ mbits
            BY[:, d] = sub(BX[:, d])
        add = lambda x, y: ((x.astype(np.uint64) + y) & 0xFFFFFFFF).astype(np.uint32)
        wraps = lambda x: int(((x & 0x80008000) != 0).sum())
        Tp = partner(T, ph)
        Z = V3.pk_add(V3.swap_halves(T), BY) if Tp is None else add(Tp, BY)
        X = add(T, BX)
        self.carries += wraps(X) + wraps(Z)
        if self.guard:                                        # the u8 wrap: bit 15 of a half
            X, Z = X & 0x7FFF7FFF, Z & 0x7FFF7FFF
        self.M = V3.pk_min(X, Z)
        self.tr += 1
        if self.tr % 8 == 6:
            slot = ((self.tr - 6) // 8) % RING
            for l in range(NL):
                for d in range(ND):
                    for h in range(2):
                        s = V3.rotl6(int(POS[l, d, h]), self.tr)
                        self.ring[slot, s] = (int(self.M[l, d]) >> (16 * h)) & 0xFF

    def traceback(self, Mt, T, cnt, look):
        # the v3 traceback over this layout's positions
        best = None
        for l in range(NL):
            for d in range(ND):
                for h in range(2):
                    half = (int(Mt[l, d]) >> (16 * h)) & 0xFFFF
                    s = V3.rotl6(int(POS[l, d, h]), T)
                    m = ((half >> 7) & 0xFE) | ((half >> ((T + 1) % 8)) & 1)
                    n = (T - 6) % 8
                    pad = ((half & ((1 << n) - 1)) << (8 - n)) & 0xFF
                    key = ((m << 8) | (4 * s)) & 0xFFFF
                    key = key - 65536 if key >= 32768 else key
                    if best is None or key < best[0]:
                        best = (key, s, pad)
        _, s, pad = best
        Z = s | (V3.bitrev(pad, 8) << 6)
        c_hi = T - look
        c_first = c_hi - cnt + 8
        C0 = T - ((T - 6) % 8)
        sc = (Z >> (T - C0)) & 63
        blocks = {}
        C = C0
        while C >= c_first:
            b = int(self.ring[((C - 6) // 8) % RING, sc])
            if C <= c_hi:
                blocks[C] = b
            sc = V3.bitrev(b & 63, 6)
            C -= 8
        return [blocks[c] for c in range(c_first, c_hi + 1, 8)]


def decode(soft, frame_len, code_rate, guard=True, stats=None):
    """Model of one packet through the 8-lane layout (vit3_model.decode's driver loop).
    guard=False runs the guard-free column everywhere; `stats` (a dict) then receives the
    low-half carry count (0 whenever no metric wrapped) and the smallest H_min the rate-3/4
    body checks saw at columns 6, 12, 18 of each 24-column body."""
    P = Packet(frame_len, code_rate)
    P.guard = guard
    kinds = V3.KINDS[code_rate]
    G = {0: 2, 1: 3, 2: 4}[code_rate]
    soft = np.asarray(soft, np.int64)
    pend = None
    for g in range(soft.size // G):
        s = soft[g * G:(g + 1) * G]
        args = [(s[0], s[1])] + [(v, 0) for v in s[2:]]
        for k, kind in enumerate(kinds):
            P.step5(kind, *args[k])
            if stats is not None and P.tr % 24 in (6, 12, 18):
                h = 2 * min(int(((P.M >> 8) & 0x7F).min()), int(((P.M >> 24) & 0x7F).min()))
                stats["max_check_hmin"] = max(stats.get("max_check_hmin", 0), h)
        if P.tr % 8 == 0:
            P.normalize()
        if P.tr >= P.end:
            if pend is not None:
                P.out += P.traceback(*pend)
                pend = None
            cnt = P.end - P.ob - 6
            if cnt:
                P.out += P.traceback(P.M, P.tr, cnt, P.tr - P.end)
            P.done = True
            break
        if P.tr >= P.ob + 286:
            assert pend is None
            pend = (P.M.copy(), P.tr, 256, 24 + (P.tr - P.ob - 286) % 8)
            P.ob += 256
        if pend is not None and P.tr % 24 == 0:
            P.out += P.traceback(*pend)
            pend = None
    if pend is not None:
        P.out += P.traceback(*pend)
    if stats is not None:
        stats["carries"] = stats.get("carries", 0) + P.carries
    return np.array(P.out, np.uint8)


def signal_header_bits(soft48):
    """k_signal_vit's SIGNAL decode (zrx_kernels.hip sig_header_bits) on this layout: 24 rate-1/2
    columns, normalize after 8, 16, 24, pads stored at columns 14 and 22; the 18 header bits
    (bits 6..23 of Viterbi_sig11's traceback word, viterbicore.hpp:272-315) are the decisions
    of columns 7..24 along the winner's path: 23, 24 from its newest pad bits, 15..22 and 7..14
    from the stored pads."""
    soft48 = np.asarray(soft48, np.int64)
    P = Packet(3, 0)
    P.guard = False
    for c in range(1, 25):
        P.step5(V3.FULL, int(soft48[2 * c - 2]), int(soft48[2 * c - 1]))
        if P.tr % 8 == 0:
            P.normalize()
    assert P.carries == 0
    best = None
    for l in range(NL):
        for d in range(ND):
            for h in range(2):
                half = (int(P.M[l, d]) >> (16 * h)) & 0xFFFF
                m = ((half >> 7) & 0xFE) | ((half >> 1) & 1)
                key = (((m << 8) | (4 * int(POS[l, d, h]))) & 0xFFFF) ^ 0x8000   # 24 mod 6 = 0: state = position
                cand = (key << 16) | (half & 3)
                best = cand if best is None else min(best, cand)
    s0, pad = (best >> 18) & 63, best & 3
    s22 = (s0 >> 2) | ((pad >> 1) << 4) | ((pad & 1) << 5)
    b22 = int(P.ring[(22 - 6) // 8, s22])
    b14 = int(P.ring[(14 - 6) // 8, V3.bitrev(b22 & 63, 6)])
    return b14 | (b22 << 8) | (pad << 16)
