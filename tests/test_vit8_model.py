"""CPU check of the 8-lane Viterbi row layout (tests/vit8_model.py) against the reference
golden frames and the oracle (integer work: exact)."""
import numpy as np
import pytest

from tests import vit8_model as V


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
                elif src[0] == "mk":
                    assert a ^ b == ((4 ^ 12) | ((4 ^ 12) << 16)), (ph, d, l)
                else:                                   # complement: P byte 3 - k, marker as src[2] says
                    for h in range(2):
                        ka, kb = (a >> (16 * h + 8)) & 3, (b >> (16 * h + 8)) & 3
                        ma, mb = (a >> (16 * h)) & 0xFF, (b >> (16 * h)) & 0xFF
                        assert ka == 3 - kb, (ph, d, l)
                        assert (ma != mb) == bool(src[2]), (ph, d, l)


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


@pytest.mark.parametrize("cr", [0, 1, 2])
def test_guard_free_columns(golden, oracle, cr):
    """The guard-free column (zrx_viterbi3.hpp "Guard-free columns"): on the reference frames,
    the adversarial fixture, noisy and pure-noise frames, no low-half add carries into bit 16
    (no metric wrap) and the output equals the guarded model's, i.e. the reference's.  Clean
    and noisy rate-3/4 frames keep every body check's H_min far below the 115 bound; pure
    noise passes it (the kernel then redoes such bodies with the guard)."""
    from tests.golden import synth
    g = golden["ref_viterbi"]
    cases, so, oo = g["vit_cases"], g["vit_soft_off"], g["vit_out_off"]
    short = [i for i, c in enumerate(cases) if c[1] <= 333 and c[0] == cr]
    for i in short[:4]:
        _, fl, _ = cases[i]
        st = {}
        got = V.decode(g["vit_soft"][so[i]:so[i + 1]], int(fl), cr, guard=False, stats=st)
        assert st["carries"] == 0
        assert (got == g["vit_out"][oo[i]:oo[i + 1]]).all()
    st = {}
    got = V.decode(g["vit_adv_soft"], 1000, cr, guard=False, stats=st)
    exp = g[f"vit_adv_out_{cr}"]
    assert st["carries"] == 0 and (got[:exp.size] == exp).all()
    for noise, seed in ((3, 11), (-1, 12), (-1, 13)):
        s = synth.viterbi_soft(cr, 300, noise, seed=seed)
        st = {}
        got = V.decode(s, 300, cr, guard=False, stats=st)
        assert st["carries"] == 0 and (got == oracle.viterbi_decode(s, 300, cr)).all()
        if cr == 2 and noise >= 0:
            assert st["max_check_hmin"] <= 115


def test_signal_rows_model(golden, oracle):
    """The SIGNAL decode on 8-lane rows (k_signal_vit) against the reference's SIGNAL vectors
    and the oracle's Viterbi_sig11 on random and near-clean soft values."""
    g = golden["ref_viterbi"]
    for s, exp in list(zip(g["sig_soft"], g["sig_bits"]))[::4]:
        hb = V.signal_header_bits(s)
        assert hb.to_bytes(3, "little") == bytes(exp)
    rng = np.random.default_rng(21)
    for i in range(120):
        if i % 2:
            s = rng.integers(0, 8, 48)
        else:
            s = np.clip(np.where(rng.integers(0, 2, 48) == 1, 7, 0) + rng.integers(-3, 4, 48), 0, 7)
        ref = int.from_bytes(bytes(oracle.viterbi_sig(s.astype(np.int8))), "little") & 0x3FFFF
        assert V.signal_header_bits(s) == ref
