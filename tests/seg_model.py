"""Numpy model of k_viterbi3's trellis segments (zrx_viterbi3.hpp "Trellis segments"): a frame
decoded as nseg segments, each from its own start column, with the seam check and the fix
pass, restated on the brick's own state (64 u8 metrics, survivor words) rather than the
kernel's packed layout.  tests/test_seg_model.py checks it against the oracle's unsplit
decode (oracle/ziria_oracle.c zo_vit_decode = csrc/sora_ext_viterbi.cpp:66-153), so the
seam argument is proven on the CPU before the kernel runs it.

Geometry (same formulas as v3::seg_start / seg_count / seg_stop), warm-up W = 256 (mixed
batches) or 136 (uniform batches, v3::kSegWarmUni):
  J_k = 768 * round(k E / (nseg 768)) + 256   first output bit of segment k (k >= 1)
  S_k = J_k - W                                segment k's first column (S_0 = 0)
  C_k = S_k + W - 16                           seam column: both sides' metrics compared here
  segment k - 1 stops at J_k + 30              (its window at ob = J_k - 256 has then fired)
"""
import numpy as np

UNIT, WARM, CMP, MAX_SEG, MIN_SEG, MIN_CUT, MAX_END = 768, 256, 240, 8, 1536, 1024, 1 << 24
WARM_UNI = 136
PREFIX, LOOK, DEPTH = 6, 24, 256

_S = np.arange(64)
_P0 = _S >> 1
_P1 = _P0 | 32
_X = _S & 1


def _bit(v, b):
    return (v >> b) & 1


def _ea(p, x):
    return x ^ _bit(p, 1) ^ _bit(p, 2) ^ _bit(p, 4) ^ _bit(p, 5)


def _eb(p, x):
    return x ^ _bit(p, 0) ^ _bit(p, 1) ^ _bit(p, 2) ^ _bit(p, 5)


_A0, _A1, _B0, _B1 = _ea(_P0, _X), _ea(_P1, _X), _eb(_P0, _X), _eb(_P1, _X)


def _bm(v, e):
    return np.where(e, 14 - 2 * v, 2 * v)


def seg_start(E, nseg, k, warm=WARM):
    return 0 if k == 0 else UNIT * ((2 * k * E + nseg * UNIT) // (2 * nseg * UNIT)) + WARM - warm


def seg_count(E, cols, L, min_len=MIN_SEG):
    """v3::seg_count: min_len MIN_SEG for a mixed batch, MIN_CUT for a uniform one."""
    if cols < E or E > MAX_END or E < 2 * min_len or L == 0:
        return 1
    n = (cols + L - 1) // L
    n = min(n, E // min_len)
    return min(max(n, 1), MAX_SEG)


def seg_stop(E, cols, nseg, k, warm=WARM):
    return seg_start(E, nseg, k + 1, warm) + warm + 30 if k + 1 < nseg else cols


def order_place(pos, nfull, ncu, rows=32):
    """v3::order_place: sorted position -> row slot, whole blocks snake over ncu CUs."""
    b = pos // rows
    if b >= nfull:
        return pos
    r, c = divmod(b, ncu)
    base = r * ncu
    m = min(ncu, nfull - base)
    return ((base + m - 1 - c) if r & 1 else b) * rows + pos % rows


def rank_place(r, nfull, ncu, rows=32):
    """v3::rank_place: block rank (0 = longest) -> block slot (blocks dealt to CU slot mod ncu)."""
    if nfull <= ncu:
        return r
    if nfull <= 2 * ncu:
        n2 = nfull - ncu
        alone = ncu - n2
        if r < alone:
            return ncu - 1 - r
        q = r - alone
        return q if q < n2 else ncu + (2 * n2 - 1 - q)
    return order_place(r * rows, nfull, ncu, rows) // rows


def std_init():
    m = np.full(64, 48, np.int64)
    m[0] = 0
    return m


def _groups(cr):
    """(soft values per group, steps of a group as (soft index a, soft index b, use))"""
    if cr == 0:
        return 2, [(0, 1, 3)]
    if cr == 1:
        return 3, [(0, 1, 3), (2, 0, 1)]
    return 4, [(0, 1, 3), (2, 0, 1), (3, 0, 2)]


def cols_of(cr, n):
    G, st = _groups(cr)
    return (n // G) * len(st)


def decode_range(soft, cr, fl, S, m0, ob0, stop, dump_cols=(), cmp=None):
    """The brick loop from column S (a group boundary) with metrics m0 and output base ob0,
    until the group end at or after `stop`.  Returns (bytes {index: value}, dumps {column:
    metrics}, stop).  cmp(tr, m) -> new stop or None: called at each dump column."""
    soft = np.asarray(soft).astype(np.int64)
    G, steps = _groups(cr)
    E = 8 * fl + PREFIX
    m = np.asarray(m0, np.int64).copy()
    surv = {}
    out, dumps = {}, {}
    tr, ob = S, ob0
    i = (S // len(steps)) * G
    while i + G <= soft.size and tr < stop:
        for ia, ib, use in steps:
            a, b = soft[i + ia], soft[i + ib]
            b0 = np.zeros(64, np.int64)
            b1 = np.zeros(64, np.int64)
            if use & 1:
                b0 += _bm(a, _A0); b1 += _bm(a, _A1)
            if use & 2:
                v = a if use == 2 else b
                b0 += _bm(v, _B0); b1 += _bm(v, _B1)
            r0 = ((m[_P0] + b0) & 0xFF) & 0xFE
            r1 = ((m[_P1] + b1) & 0xFF) | 1
            m = np.minimum(r0, r1)
            tr += 1
            surv[tr] = m & 1
        i += G
        if tr % 8 == 0:
            m = (m - (m.min() & 0xFE)) & 0xFF
        if tr in dump_cols:
            dumps[tr] = m.copy()
            if cmp is not None:
                s2 = cmp(tr, m)
                if s2 is not None:
                    stop = min(stop, s2)
        cnt = look = 0
        if tr >= E:
            cnt, look = E - ob - PREFIX, tr - E
        elif tr >= ob + DEPTH + LOOK + PREFIX:
            cnt, look = DEPTH, LOOK + (tr - (ob + DEPTH + LOOK + PREFIX)) % 8
        if cnt:
            key = ((m << 8) | (4 * _S)).astype(np.int64) & 0xFFFF
            key = np.where(key >= 0x8000, key - 0x10000, key)
            st = int((key.min() >> 2) & 0x7F)
            t = tr
            for _ in range(look):
                t -= 1
                st = ((st >> 1) & 0x3F) | (int(surv[t][(st >> 1) & 0x3F]) << 6)
            nb = cnt >> 3
            for byte in range(nb - 1, -1, -1):
                oc = 0
                for _ in range(8):
                    oc = (oc << 1) | ((st >> 6) & 1)
                    t -= 1
                    st = ((st >> 1) & 0x3F) | (int(surv[t][(st >> 1) & 0x3F]) << 6)
                out[ob // 8 + byte] = oc
            ob += cnt
    return out, dumps, stop


def segmented_decode(soft, cr, fl, nseg, warm=WARM):
    """Pass 1 over the nseg segments, the seam check, the fix pass; returns (bytes, number
    of fix rows run)."""
    E = 8 * fl + PREFIX
    cmpc = warm - 16
    cols = cols_of(cr, len(soft))
    out = {}
    A, B = {}, {}                                        # seam j: side A (segment j-1), side B (segment j)
    for k in range(nseg):
        S = seg_start(E, nseg, k, warm)
        dc = set()
        if k:
            dc.add(S + cmpc)
        if k + 1 < nseg:
            dc.add(seg_start(E, nseg, k + 1, warm) + cmpc)
        o, d, _ = decode_range(soft, cr, fl, S, std_init() if k == 0 else np.zeros(64, np.int64),
                               0 if k == 0 else S + warm, seg_stop(E, cols, nseg, k, warm), dc)
        out.update(o)
        if k:
            B[k] = d[S + cmpc]
        if k + 1 < nseg:
            A[k + 1] = d[seg_start(E, nseg, k + 1, warm) + cmpc]
    fixes = 0
    bad = [j for j in range(1, nseg) if ((A[j] ^ B[j]) & 0xFE).any()]
    if bad:
        # one fix row from the first disagreeing seam, from segment ks - 1's state; it may stop
        # only at a seam past the last disagreeing one whose start state it reproduces
        ks, kl = bad[0], bad[-1]
        fixes = 1
        S = seg_start(E, nseg, ks, warm) + cmpc
        cmp_cols = {seg_start(E, nseg, j, warm) + cmpc: j for j in range(kl + 1, nseg)}

        def cmp(tr, m):
            j = cmp_cols[tr]
            if not ((m ^ B[j]) & 0xFE).any():
                return seg_start(E, nseg, j, warm) + warm + 30
            return None
        o, _, _ = decode_range(soft, cr, fl, S, A[ks], S + warm - cmpc, cols, set(cmp_cols), cmp)
        out.update(o)
    n = max(out) + 1 if out else 0
    return np.array([out[i] for i in range(n)], np.uint8), fixes
