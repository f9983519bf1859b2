"""Trellis segments on the CPU (tests/seg_model.py): the segment geometry's invariants, and a
frame decoded as segments with the seam check and the fix pass equals the oracle's unsplit
decode bit for bit, at every rate, clean and noisy, including pure-noise frames whose seams
disagree (so the fix pass really runs)."""
import numpy as np
import pytest

from tests import seg_model as SM
from tests.golden import synth


@pytest.mark.parametrize("warm", [SM.WARM, SM.WARM_UNI])
def test_geometry_invariants(warm):
    for fl in list(range(384, 5000, 37)) + [2050, 4095]:
        E = 8 * fl + 6
        for cr in (0, 1, 2):
            K = (24, 32, 36)[cr]                             # decoded bits per 48 soft values
            cols = -(-E // K) * K
            for nseg in range(2, min(SM.MAX_SEG, E // SM.MIN_CUT) + 1):
                S = [SM.seg_start(E, nseg, k, warm) for k in range(nseg)]
                assert S[0] == 0 and all(b > a for a, b in zip(S, S[1:]))
                for k in range(1, nseg):
                    J = S[k] + warm                          # first output bit: a window boundary
                    assert J % 768 == 256 and S[k] % 24 == 0 and S[k] > 0
                    assert J + 64 <= E                       # window J_k - 256 fires before the frame end
                    assert (S[k] + warm - 16) % 24 == 0      # the seam column is a body end
                    assert S[k] + warm - 16 > S[k - 1]       # ... inside segment k - 1
                for k in range(nseg):
                    assert SM.seg_stop(E, cols, nseg, k, warm) > S[k] + warm - 16


def test_row_bound():
    """sum of segments <= batch columns / L' + packets, L' = 9/8 max(1024, columns / (64 ncu))
    (uniform batch) or 11/8 L (mixed, v3::kSegMixNum), L = max(1536, columns / (64 ncu)): within
    the grid of k_viterbi3's
    planned launch (zrx_api.hip plan_rows_max), for mixed and uniform batches."""
    rng = np.random.default_rng(3)
    ncu, mix = 256, 11
    r = 64 * 8 * ncu // min(mix, 8)
    for it in range(300):
        n = int(rng.integers(1, 20000))
        if it % 2:                                       # uniform: one frame length for all
            fl = np.full(n, int(rng.integers(1, 4096)))
            cols = 8 * fl + 6 + int(rng.integers(0, 300))
        else:
            fl = rng.integers(1, 4096, n)
            cols = 8 * fl + 6 + rng.integers(0, 300, n)
        E = 8 * fl + 6
        T = int(np.sum(cols))
        L0 = -(-T // (64 * ncu))
        L, Lu = max(SM.MIN_SEG, L0), max(SM.MIN_CUT, L0)
        Lq = Lu + Lu // 8 if it % 2 else max(L * mix // 8, SM.MIN_SEG)
        mn = SM.MIN_CUT if it % 2 else SM.MIN_SEG
        rows = sum(SM.seg_count(int(e), int(c), Lq, mn) for e, c in zip(E, np.broadcast_to(cols, E.shape)))
        assert rows <= min(n + r + r // 256 + 64, n * SM.MAX_SEG), (it, n, rows)


def test_rank_place():
    """The ranked block placement of a mixed batch (v3::rank_place, restated in seg_model) is a
    permutation of the whole blocks; up to two rounds, the longest blocks sit alone on the CUs
    the second round leaves free (the partial last block's CU getting the shortest of them),
    and every other CU holds ranks summing to the same total (longest with shortest)."""
    for ncu in (2, 3, 8, 256):
        for nfull in list(range(1, 3 * ncu + 3)) if ncu < 256 else (1, 255, 256, 257, 300, 496, 511, 512, 513, 900):
            slots = [SM.rank_place(r, nfull, ncu) for r in range(nfull)]
            assert sorted(slots) == list(range(nfull)), (ncu, nfull)
            if ncu < nfull <= 2 * ncu:
                n2 = nfull - ncu
                cu = {}
                for r, s in enumerate(slots):
                    cu.setdefault(s % ncu, []).append(r)
                alone = [v for v in cu.values() if len(v) == 1]
                pairs = [v for v in cu.values() if len(v) == 2]
                assert len(pairs) == n2 and len(alone) == ncu - n2
                if alone:                                      # the longest alone
                    assert max(v[0] for v in alone) < min(min(v) for v in pairs)
                assert len({sum(v) for v in pairs}) == 1
                if ncu - n2 > 0:                               # CU n2 (the partial block's) gets the shortest alone
                    assert cu[n2] == [ncu - n2 - 1]


CASES = [(cr, fl, noise, nseg) for cr in (0, 1, 2) for fl, noise, nseg in
         [(400, 0, 2), (700, 3, 3), (1100, 2, 5), (700, -1, 3), (1100, -1, 5),
          (500, 2, 3), (500, -1, 3)]]      # (500: E / 3 = 1335 >= kMinCut, a one-unit middle segment)


@pytest.mark.parametrize("warm", [SM.WARM, SM.WARM_UNI])
@pytest.mark.parametrize("cr,fl,noise,nseg", CASES)
def test_segmented_equals_oracle(oracle, cr, fl, noise, nseg, warm):
    s = synth.viterbi_soft(cr, fl, noise, seed=100 * cr + fl + noise)
    exp = oracle.viterbi_decode(s, fl, cr)
    got, fixes = SM.segmented_decode(s, cr, fl, nseg, warm)
    assert got.size == exp.size == fl
    assert (got == exp).all()
    if noise >= 0:
        assert fixes == 0                                # clean frames converge in the warm-up


@pytest.mark.parametrize("warm", [SM.WARM, SM.WARM_UNI])
def test_pure_noise_exercises_fix(oracle, warm):
    """Pure-noise frames: some seam disagrees, the fix row re-decodes from it, still exact."""
    fixes = 0
    for seed in range(6):
        s = synth.viterbi_soft(2, 900, -1, seed=seed)
        got, f = SM.segmented_decode(s, 2, 900, 4, warm)
        assert (got == oracle.viterbi_decode(s, 900, 2)).all(), seed
        fixes += f
    assert fixes > 0


@pytest.mark.parametrize("warm", [SM.WARM, SM.WARM_UNI])
def test_pure_noise_many_seams(oracle, warm):
    """Long pure-noise frames cut into 8: several seams disagree, not always next to each
    other (a fix row that stopped at the first seam it agrees with would leave a later
    disagreeing segment in place)."""
    for seed in (7041, 41, 42):                          # 7041: seams 1, 4, 6, 7 disagree
        s = synth.viterbi_soft(2, 2035, -1, seed=seed)
        got, _ = SM.segmented_decode(s, 2, 2035, 8, warm)
        assert (got == oracle.viterbi_decode(s, 2035, 2)).all(), seed
