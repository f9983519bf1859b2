"""Executable model of the v3 Viterbi kernel's data layout (test infrastructure).

This is NOT the oracle: it restates, in numpy, exactly what k_viterbi3
(ziria_amd/csrc/zrx_viterbi3.hpp) does per lane, so that the layout tricks can be checked
against the oracle on the CPU before they run on the GPU.  One packet = 16 lanes x 2
dwords x 2 16-bit halves = 64 trellis positions.

Half layout: [H = the reference's u8 metric with its marker bit cleared (always even)]
             [pad: bit 7 = marker of the last column (= the decision), bits 6..0 = the
              previous 7 decisions along the survivor path (register exchange)]
Position p holds state rotl6(p, t mod 6) after t columns (labels rotate, positions stay);
its butterfly partner at column t is p ^ (1 << (5 - t mod 6)).
Reference semantics: csrc/sora_ext_viterbi.cpp:66-153 over csrc/viterbicore.hpp:105-239.
"""
import numpy as np

RING = 39                       # snapshot slots (8 columns each) per packet
FULL, AONLY, BONLY = 0, 1, 2
KINDS = {0: [FULL], 1: [FULL, AONLY], 2: [FULL, AONLY, BONLY]}
XOR_OF_BIT = {2: 1, 3: 2, 4: 15, 5: 8}   # position bit -> lane xor (DPP qp / qp / row_mirror / row_ror:8)


def rotl6(x, k):
    k %= 6
    x &= 63
    return ((x << k) | (x >> (6 - k))) & 63 if k else x


def lane_of(p):
    l = 0
    for b, x in XOR_OF_BIT.items():
        if (p >> b) & 1:
            l ^= x
    return l


def pos_of(lane, d, h):
    l0, l1, l2, l3 = (lane >> 0) & 1, (lane >> 1) & 1, (lane >> 2) & 1, (lane >> 3) & 1
    b4 = l2
    b2, b3, b5 = l0 ^ b4, l1 ^ b4, l3 ^ b4
    return h | (d << 1) | (b2 << 2) | (b3 << 3) | (b4 << 4) | (b5 << 5)


def bitrev(x, n):
    r = 0
    for i in range(n):
        r |= ((x >> i) & 1) << (n - 1 - i)
    return r


POS = np.array([[[pos_of(l, d, h) for h in range(2)] for d in range(2)] for l in range(16)])
assert sorted(POS.ravel().tolist()) == list(range(64))
assert all(lane_of(pos_of(l, d, h)) == l for l in range(16) for d in range(2) for h in range(2))


def selectors():
    """sel[phase][lane][dword]: v_perm selector building [BM_hi][bm_hi<<7][BM_lo][bm_lo<<7]."""
    sel = np.zeros((6, 16, 2), np.uint32)
    for ph in range(6):
        for l in range(16):
            for d in range(2):
                w = 0
                for h in range(2):
                    j = rotl6(int(POS[l, d, h]), ph)
                    bm = (j >> 5) & 1
                    A = ((j >> 1) ^ (j >> 2) ^ (j >> 4)) & 1
                    B = (j ^ (j >> 1) ^ (j >> 2)) & 1
                    w |= (4 if bm else 12) << (16 * h)
                    w |= (2 * A + B) << (16 * h + 8)
                sel[ph, l, d] = w
    return sel


SEL = selectors()


def c_words(k):
    """Per-lane BY = C - BX constants: per half (k + bm) << 8, so that BY keeps BX's marker
    (both candidates of one source state carry that state's branch index) while its branch
    metric is the complement k - BM (k = 28 for a full step, 14 for a punctured one)."""
    c = np.zeros((6, 16, 2), np.uint32)
    for ph in range(6):
        for l in range(16):
            for d in range(2):
                for h in range(2):
                    j = rotl6(int(POS[l, d, h]), ph)
                    c[ph, l, d] |= (k + ((j >> 5) & 1)) << (16 * h + 8)
    return c


CW = {28: c_words(28), 14: c_words(14)}


def perm(s0, s1, sel):
    """v_perm_b32 D, S0, S1, sel: byte i of D = byte sel_i of {S0:S1} (S1 = low dword)."""
    s0 = np.asarray(s0, np.uint64)
    s1 = np.asarray(s1, np.uint64)
    src = (s0 << np.uint64(32)) | s1
    out = np.zeros(np.broadcast(s0, s1, sel).shape, np.uint64)
    for i in range(4):
        b = (np.asarray(sel, np.uint64) >> np.uint64(8 * i)) & np.uint64(0xFF)
        v = (src >> (np.uint64(8) * (b & np.uint64(7)))) & np.uint64(0xFF)
        v = np.where(b == 12, np.uint64(0), v)
        out |= v << np.uint64(8 * i)
    return out.astype(np.uint32)


def pk(op, a, b):
    a = np.asarray(a, np.uint32)
    b = np.asarray(b, np.uint32)
    lo = op(a & 0xFFFF, b & 0xFFFF) & 0xFFFF
    hi = op(a >> 16, b >> 16) & 0xFFFF
    return (lo | (hi << 16)).astype(np.uint32)


def pk_add(a, b):
    return pk(lambda x, y: x + y, a, b)


def pk_sub(a, b):
    return pk(lambda x, y: x - y, a, b)


def pk_min(a, b):
    return pk(np.minimum, a, b)


def swap_halves(a):
    return ((a >> 16) | (a << 16)).astype(np.uint32)


def p_word(kind, a, b):
    a2 = (2 * (a & 7)) * 0x01010101
    b2 = (2 * (b & 7)) * 0x01010101
    if kind == FULL:
        return ((a2 ^ 0x0E0E0000) + (b2 ^ 0x0E000E00)) & 0xFFFFFFFF
    if kind == AONLY:
        return a2 ^ 0x0E0E0000
    return a2 ^ 0x0E000E00


class Packet:
    def __init__(self, frame_len, code_rate):
        self.fl, self.cr = frame_len, code_rate
        st = np.where(POS == 0, 0, 48).astype(np.uint32)
        self.M = ((st[..., 1] << 24) | (st[..., 0] << 8)).astype(np.uint32)   # [16, 2]
        self.ring = np.zeros((RING, 64), np.uint8)
        self.tr = 0
        self.ob = 0
        self.end = 8 * frame_len + 6
        self.out = []
        self.done = False
        self.v5 = False

    def step(self, kind, a, b):
        ph = self.tr % 6
        M = self.M
        S = M >> 1
        M1 = ((S & 0x00FF00FF) | (M & 0xFF00FF00)).astype(np.uint32)
        BX = perm(0x80808080, p_word(kind, a, b), SEL[ph])
        BY = ((CW[28 if kind == FULL else 14][ph].astype(np.int64) - BX) & 0xFFFFFFFF).astype(np.uint32)
        X = pk_add(M1, BX)
        Y = pk_add(M1, BY)
        if ph <= 3:
            Yp = Y[np.arange(16) ^ XOR_OF_BIT[5 - ph]]
        elif ph == 4:
            Yp = Y[:, ::-1]
        else:
            Yp = swap_halves(Y)
        self.M = pk_min(X, Yp)
        self.tr += 1
        if self.tr % 8 == 6:                                # snapshot column
            slot = ((self.tr - 6) // 8) % RING
            for l in range(16):
                for d in range(2):
                    for h in range(2):
                        s = rotl6(int(POS[l, d, h]), self.tr)
                        self.ring[slot, s] = (int(self.M[l, d]) >> (16 * h)) & 0xFF

    def step4(self, kind, a, b):
        """v4 column: one v_add_u32 per candidate instead of v_pk_add_u16, the cross
        candidate added straight from the partner lane (v_add_u32_dpp) with the complement
        branch metric C - BX of this position (the partner state j ^ 32 has the same expected
        bits and the other marker), pads cleared after each snapshot.  A 32-bit add carries
        out of half 0 into bit 0 of half 1's pad when H0 wraps; that bit is 0 at every
        non-snapshot column (cleared 1..7 columns earlier) and is never read, and the
        snapshot column itself uses exact packed adds."""
        ph = self.tr % 6
        c = self.tr + 1                                   # column being computed
        M = self.M
        if c % 8 == 7:                                    # first column after a snapshot
            T = (M & 0xFF00FF00).astype(np.uint32)
        else:
            T = (((M >> 1) & 0x00FF00FF) | (M & 0xFF00FF00)).astype(np.uint32)
        if c % 8 != 7 and c % 8 != 6:
            assert ((T >> 16) & 1).max() == 0, "half-1 guard bit set at a 32-bit add"
        BX = perm(0x80808080, p_word(kind, a, b), SEL[ph])
        C = 0x1C801C80 if kind == FULL else 0x0E800E80
        BY = ((C - BX.astype(np.int64)) & 0xFFFFFFFF).astype(np.uint32)
        exact = c % 8 == 6
        add = pk_add if exact else (lambda x, y: ((x.astype(np.uint64) + y) & 0xFFFFFFFF).astype(np.uint32))
        if ph <= 3:
            Tp = T[np.arange(16) ^ XOR_OF_BIT[5 - ph]]
            Z = add(Tp, BY)
        elif ph == 4:
            Z = add(T[:, ::-1], BY)
        else:
            Z = pk_add(swap_halves(T), BY)
        X = add(T, BX)
        self.M = pk_min(X, Z)
        self.tr += 1
        if self.tr % 8 == 6:
            slot = ((self.tr - 6) // 8) % RING
            for l in range(16):
                for d in range(2):
                    for h in range(2):
                        s = rotl6(int(POS[l, d, h]), self.tr)
                        self.ring[slot, s] = (int(self.M[l, d]) >> (16 * h)) & 0xFF

    def step5(self, kind, a, b):
        """v5 column: no pad shift.  The column with cycle phase k = (c + 1) % 8 (c = the
        column being computed; k = 7 is the snapshot column) writes its marker at bit k + 1
        of each half, so a half is [H >> 1 (bits 15..9)][decisions of the cycle, bits 8..1,
        oldest lowest][bit 0: carry guard].  Bits above the marker are still 0 in both
        candidates (cleared at k = 0), so the marker decides ties exactly as the brick's
        metric LSB (viterbicore.hpp:105-147); a snapshot byte is bits 8..1.  The 32-bit adds
        carry out of half 0 into bit 16 only, which one AND per column clears (k = 0: the AND
        also clears the cycle's history).  At k = 7 the marker is bit 8, the H byte's LSB
        (H is even): BX = [BM][bm<<7] + (its low byte) = [BM + bm][0]."""
        ph = self.tr % 6
        c = self.tr + 1
        k = (c + 1) % 8
        M = self.M
        T = (M & (0xFE00FE00 if k == 0 else 0xFFFEFFFF)).astype(np.uint32)
        mk = 2 << k
        src0 = 0x80808080 if k == 7 else mk * 0x01010101
        BX = perm(src0, p_word(kind, a, b), SEL[ph])
        if k == 7:
            BX = (BX + (BX & 0x00FF00FF)).astype(np.uint32)
        K = 28 if kind == FULL else 14
        C = ((K + 1) << 8) * 0x00010001 if k == 7 else ((K << 8) | mk) * 0x00010001
        BY = ((C - BX.astype(np.int64)) & 0xFFFFFFFF).astype(np.uint32)
        add = lambda x, y: ((x.astype(np.uint64) + y) & 0xFFFFFFFF).astype(np.uint32)
        if ph <= 3:
            Z = add(T[np.arange(16) ^ XOR_OF_BIT[5 - ph]], BY)
        elif ph == 4:
            Z = add(T[:, ::-1], BY)
        else:
            Z = pk_add(swap_halves(T), BY)
        X = add(T, BX)
        self.M = pk_min(X, Z)
        self.tr += 1
        if self.tr % 8 == 6:
            slot = ((self.tr - 6) // 8) % RING
            for l in range(16):
                for d in range(2):
                    for h in range(2):
                        s = rotl6(int(POS[l, d, h]), self.tr)
                        self.ring[slot, s] = (int(self.M[l, d]) >> (16 * h + 1)) & 0xFF

    def normalize(self):
        H = np.concatenate([(self.M & 0xFFFF).ravel(), (self.M >> 16).ravel()]) >> 8
        mn = int(H.min())
        self.M = pk_sub(self.M, np.uint32((mn << 8) | (mn << 24)))

    def traceback(self, Mt, T, cnt, look):
        best = None
        for l in range(16):
            for d in range(2):
                for h in range(2):
                    half = (int(Mt[l, d]) >> (16 * h)) & 0xFFFF
                    s = rotl6(int(POS[l, d, h]), T)
                    if self.v5:                           # marker of column T at bit (T+1)%8 + 1
                        m = ((half >> 8) & 0xFE) | ((half >> ((T + 1) % 8 + 1)) & 1)
                        n = (T - 6) % 8                   # decisions since the snapshot, bits n..1
                        pad = (((half >> 1) & ((1 << n) - 1)) << (8 - n)) & 0xFF
                        half = (half & 0xFF00) | pad       # the v3 pad form
                    else:
                        m = (half >> 8) | ((half >> 7) & 1)
                    key = ((m << 8) | (4 * s)) & 0xFFFF
                    key = key - 65536 if key >= 32768 else key
                    if best is None or key < best[0]:
                        best = (key, s, half & 0xFF)
        _, s, pad = best
        Z = s | (bitrev(pad, 8) << 6)
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
            sc = bitrev(b & 63, 6)
            C -= 8
        return [blocks[c] for c in range(c_first, c_hi + 1, 8)]


def decode(soft, frame_len, code_rate, v4=False):
    """Model of one packet through k_viterbi3 (whole soft buffer, 24-column bodies);
    v4 = the carry-tolerant 32-bit-add column (Packet.step4), v4 = 5 the shift-free
    ascending-marker column (Packet.step5)."""
    P = Packet(frame_len, code_rate)
    P.v5 = v4 == 5
    stepf = P.step5 if v4 == 5 else P.step4 if v4 else P.step
    kinds = KINDS[code_rate]
    G = {0: 2, 1: 3, 2: 4}[code_rate]
    soft = np.asarray(soft, np.int64)
    pend = None
    for g in range(soft.size // G):
        s = soft[g * G:(g + 1) * G]
        args = [(s[0], s[1])] + [(v, 0) for v in s[2:]]
        for k, kind in enumerate(kinds):
            stepf(kind, *args[k])
        if P.tr % 8 == 0:
            P.normalize()
        if P.tr >= P.end:
            if pend is not None:                           # a deferred window runs first
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
        if pend is not None and P.tr % 24 == 0:            # body end: run the deferred window
            P.out += P.traceback(*pend)
            pend = None
    if pend is not None:
        P.out += P.traceback(*pend)
    return np.array(P.out, np.uint8)
