"""CPU check of the 4-lane Viterbi row layout (tests/vit4_model.py) against the reference
golden frames and the oracle (integer work: exact)."""
import numpy as np
import pytest

from tests import vit4_model as V


def test_position_map_and_partners():
    assert sorted(V.POS.ravel().tolist()) == list(range(64))
    for bit, x in V.XOR_OF_BIT.items():
        for l in range(V.NL):
            for d in range(V.ND):
                for h in range(2):
                    assert V.lane_of(int(V.POS[l, d, h]) ^ (1 << bit)) == l ^ x


def test_bx_sources_hold():
    """every shared / marker-flipped branch-metric word equals the word its own selector builds"""
    for ph in range(6):
        for d in range(V.ND):
            src = V.bx_source(ph, d)
            if src[0] == "perm":
                continue
            for l in range(V.NL):
                a, b = int(V.SEL[ph, l, d]), int(V.SEL[ph, l, src[1]])
                if src[0] == "same":
                    assert a == b, (ph, d, l)
                else:
                    assert a ^ b == ((4 ^ 12) | ((4 ^ 12) << 16)), (ph, d, l)


@pytest.mark.parametrize("idx", range(0, 48, 3))
def test_model_matches_reference_frames(golden, idx):
    g = golden["ref_viterbi"]
    cases, so, oo = g["vit_cases"], g["vit_soft_off"], g["vit_out_off"]
    short = [i for i, c in enumerate(cases) if c[1] <= 333]
    i = short[idx % len(short)]
    cr, fl, _ = cases[i]
    got = V.decode(g["vit_soft"][so[i]:so[i + 1]], int(fl), int(cr))
    exp = g["vit_out"][oo[i]:oo[i + 1]]
    assert got.size == exp.size and (got == exp).all()


@pytest.mark.parametrize("cr", [0, 1, 2])
def test_model_adversarial_wrap(golden, cr):
    g = golden["ref_viterbi"]
    exp = g[f"vit_adv_out_{cr}"]
    got = V.decode(g["vit_adv_soft"], 1000, cr)
    assert (got[:exp.size] == exp).all()


def test_model_truncated_vs_oracle(oracle):
    from tests.golden import synth
    rng = np.random.default_rng(8)
    for i in range(6):
        cr = int(rng.integers(0, 3))
        fl = int(rng.integers(1, 120))
        s = synth.viterbi_soft(cr, fl, int(rng.integers(-1, 5)), seed=800 + i)
        if i % 2 == 0:
            s = s[: max(48, (s.size // 2) // 48 * 48)]
        exp = oracle.viterbi_decode(s, fl, cr)
        got = V.decode(s, fl, cr)
        assert got.size == exp.size and (got == exp).all()
