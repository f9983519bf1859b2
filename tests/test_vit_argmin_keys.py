"""CPU restatement of k_viterbi3's traceback argmin (zrx_viterbi3.hpp `traceback`): the
packed 16-bit keys with the winner's pad read afterwards pick the same state and pad as the
one-key-per-state form they replaced ([H bits 7..1 ^ sign][marker][state][0 0][pad],
unsigned minimum).  The reference's order (viterbicore.hpp:105-147 metric with the marker as
its LSB, ties to the lowest state) is what both forms encode.  Integer work: exact."""
import numpy as np
import pytest

from tests import vit3_model as V3
from tests import vit8_model as V


def rotl6(x, k):
    return V3.rotl6(int(x), int(k))


def rotr6(x, k):
    return ((int(x) * 65) >> int(k)) & 63


def old_argmin(M, T):
    """one 32-bit key per state; M: (8 lanes, 4 dwords) uint32"""
    ph, n, ms = T % 6, (T - 6) & 7, (T + 1) & 7
    best = 0xFFFFFFFF
    for l in range(8):
        for q in range(8):
            half = (int(M[l, q >> 1]) >> (16 * (q & 1))) & 0xFFFF
            st = rotl6(V.pos_of(l, q >> 1, q & 1), ph)
            pad = ((half & ((1 << n) - 1)) << (8 - n)) & 0xFF
            key = (((half & 0x7F00) << 17) | (((half >> ms) & 1) << 24) | (st << 18) | pad) ^ 0x80000000
            best = min(best, key)
    return (best >> 18) & 63, best & 0xFF


def s16(x):
    x &= 0xFFFF
    return x - 0x10000 if x & 0x8000 else x


def new_argmin(M, T):
    """two 16-bit keys per dword (signed order), then the winner's pad by a byte select"""
    ph, n, ms = T % 6, (T - 6) & 7, (T + 1) & 7
    o = 6 - ph
    r0, r1, r2 = (65 >> o) & 63, (130 >> o) & 63, (260 >> o) & 63
    sh = 8 - ms
    kb, st0s = None, []
    for l in range(8):
        st0 = ((V.pos_of(l, 0, 0) * 65) >> o) & 63
        assert st0 == rotl6(V.pos_of(l, 0, 0), ph) and r0 == rotl6(1, ph) and r2 == rotl6(4, ph)
        st0s.append(st0)
        c0 = (st0 << 2) | ((st0 ^ r0) << 18)
        rr1, rr2 = r1 * 0x40004, r2 * 0x40004
        stc = [c0, c0 ^ rr1, c0 ^ rr2, c0 ^ rr1 ^ rr2]
        for d in range(4):
            m = int(M[l, d])
            y = ((m << sh) & 0x01000100) | stc[d]
            k = (((m << 1) & 0xFE00FE00) | y) & 0xFFFFFFFF
            for h in (s16(k), s16(k >> 16)):
                kb = h if kb is None else min(kb, h)
    s0 = (kb >> 2) & 63
    pb = 0
    for l in range(8):
        q = rotr6(s0 ^ st0s[l], ph)
        pk = [(int(M[l, q2 >> 1]) >> (16 * (q2 & 1))) & 0xFF for q2 in range(8)]   # the two v_perms
        pb |= pk[q] if q < 8 else 0
    return s0, (pb << (8 - n)) & 0xFF


@pytest.mark.parametrize("seed", range(6))
def test_packed_argmin_matches_full_keys(seed):
    rng = np.random.default_rng(seed)
    for trial in range(300):
        T = int(rng.integers(6, 5000))
        if trial % 3 == 0:       # many ties: few distinct metrics
            hv = rng.integers(0, 3, size=(8, 4, 2)) << 9
            M = (hv[..., 0] | (hv[..., 1] << 16) | rng.integers(0, 1 << 9, size=(8, 4)) |
                 (rng.integers(0, 1 << 9, size=(8, 4)) << 16))
        else:                    # anything, bit 15 of each half included (ignored by both)
            M = rng.integers(0, 1 << 32, size=(8, 4), dtype=np.uint64)
        M = M.astype(np.uint64)
        assert new_argmin(M, T) == old_argmin(M, T), (seed, trial, T)
