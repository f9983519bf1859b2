"""CPU check of the v3 Viterbi kernel's layout (tests/vit3_model.py) against the reference
golden frames and the oracle: the packed-position / pad-history / snapshot-ring scheme of
ziria_amd/csrc/zrx_viterbi3.hpp must reproduce the brick bit for bit (integer work, exact)."""
import numpy as np
import pytest

from tests import vit3_model as V


def test_position_map_is_a_bijection():
    assert sorted(V.POS.ravel().tolist()) == list(range(64))
    for ph in range(4):
        bit = 5 - ph
        for l in range(16):
            for d in range(2):
                for h in range(2):
                    p = int(V.POS[l, d, h])
                    q = p ^ (1 << bit)
                    assert V.lane_of(q) == l ^ V.XOR_OF_BIT[bit]


def test_dword_selector_identities():
    """column5 derives dword 1's branch metrics from dword 0's at phases 2 and 4."""
    S = V.SEL
    assert all(S[2, l, 0] == S[2, l, 1] for l in range(16))
    assert all((S[4, l, 0] ^ S[4, l, 1]) == ((4 ^ 12) | ((4 ^ 12) << 16)) for l in range(16))


@pytest.mark.parametrize("v4", [False, True, 5])
@pytest.mark.parametrize("idx", range(0, 48, 5))
def test_model_matches_reference_frames(golden, idx, v4):
    g = golden["ref_viterbi"]
    cases, so, oo = g["vit_cases"], g["vit_soft_off"], g["vit_out_off"]
    short = [i for i, c in enumerate(cases) if c[1] <= 333]
    i = short[idx % len(short)]
    cr, fl, _ = cases[i]
    got = V.decode(g["vit_soft"][so[i]:so[i + 1]], int(fl), int(cr), v4=v4)
    exp = g["vit_out"][oo[i]:oo[i + 1]]
    assert got.size == exp.size and (got == exp).all()


@pytest.mark.parametrize("v4", [False, True, 5])
@pytest.mark.parametrize("cr", [0, 1, 2])
def test_model_adversarial_wrap(golden, cr, v4):
    g = golden["ref_viterbi"]
    exp = g[f"vit_adv_out_{cr}"]
    got = V.decode(g["vit_adv_soft"], 1000, cr, v4=v4)
    assert (got[:exp.size] == exp).all()


@pytest.mark.parametrize("v4", [False, True, 5])
def test_model_truncated_vs_oracle(oracle, v4):
    from tests.golden import synth
    rng = np.random.default_rng(5)
    for i in range(6):
        cr = int(rng.integers(0, 3))
        fl = int(rng.integers(1, 120))
        s = synth.viterbi_soft(cr, fl, int(rng.integers(-1, 5)), seed=500 + i)
        if i % 2 == 0:
            s = s[: max(48, (s.size // 2) // 48 * 48)]
        exp = oracle.viterbi_decode(s, fl, cr)
        got = V.decode(s, fl, cr, v4=v4)
        assert got.size == exp.size and (got == exp).all()
