"""The per-call externals (include/ziria_rx.h Part 1) on the host CPU, through the C-ABI of
libziria_rx.so, against the reference's own KATs, the reference-brick golden fixtures and the
oracle.  SURVEY.md §8(b) item 1 puts these symbols on "a CPU path, with the GPU used only if
batched" (ziria_amd/csrc/zrx_host.cpp), so they run here without a GPU.  Integer work: every
comparison is bit-exact."""
import numpy as np
import pytest

import ziria_amd as Z


@pytest.fixture(scope="module", autouse=True)
def _built():
    from ziria_amd import build
    build.build()


# ------------------------------------------------------------------ FFT
def test_fft64_kat(golden):
    k = golden["ref_kats"]
    assert (Z.sora_fft(k["fft64_kat_in"]) == k["fft64_kat_out"]).all()


def test_fft64_reference_vectors_per_call(golden):
    g = golden["ref_fft64"]
    for x, y in zip(g["fft_in"], g["fft_out"]):
        assert (Z.sora_fft(x) == y).all()


def test_fft64_random_and_saturating_vs_oracle(oracle):
    rng = np.random.default_rng(11)
    x = rng.integers(-32768, 32768, (600, 64, 2)).astype(np.int16)
    x[:200] = rng.choice(np.array([-32768, 32767, -1, 0], np.int16), (200, 64, 2))
    exp = oracle.fft64(x)
    for i in range(x.shape[0]):
        assert (Z.sora_fft(x[i]) == exp[i]).all(), i


def test_fft_unsupported_size_leaves_output():
    for n in (20, 100, 4096):
        x = np.ones((n, 2), np.int16)
        assert (Z.sora_fft(x) == 0).all()
    assert (Z.sora_fft_dynamic(64, np.ones((64, 2), np.int16)) == Z.sora_fft(np.ones((64, 2), np.int16))).all()


def test_fft_all_sizes_kat_per_call(golden):
    """__ext_sora_fft per call on every block of tests/libs/test_fft (all 42 sizes)."""
    g = golden["ref_fftn"]
    off = 0
    for n in g["sizes"]:
        n = int(n)
        assert (Z.sora_fft(g["kat_in"][off:off + n]) == g["kat_out"][off:off + n]).all(), n
        assert (Z.sora_fft_dynamic(n, g["kat_in"][off:off + n]) == g["kat_out"][off:off + n]).all(), n
        off += n


def test_fft_all_sizes_reference_vectors_per_call(golden):
    """The reference brick's outputs on random, saturating and small vectors of every size."""
    g = golden["ref_fftn"]
    o, per = g["vec_off"], int(g["vec_per"])
    for i, n in enumerate(g["sizes"]):
        n = int(n)
        blk = g["vec_in"][o[i * per]:o[(i + 1) * per]].reshape(per, n, 2)
        exp = g["vec_out"][o[i * per]:o[(i + 1) * per]].reshape(per, n, 2)
        for j in range(per):
            assert (Z.sora_fft(blk[j]) == exp[j]).all(), (n, j)


def test_fft_all_sizes_random_vs_oracle(oracle):
    rng = np.random.default_rng(42)
    for n in oracle.FFT_SIZES:
        x = rng.integers(-32768, 32768, (6, n, 2)).astype(np.int16)
        x[:2] = rng.choice(np.array([-32768, 32767, -1, 0, 1], np.int16), (2, n, 2))
        exp = oracle.fft_n(n, x)
        for j in range(x.shape[0]):
            assert (Z.sora_fft(x[j]) == exp[j]).all(), n


def test_v_shift_right_complex16(oracle):
    rng = np.random.default_rng(5)
    for n in (1, 3, 4, 5, 8, 13):
        for sh in (0, 1, 7, 15, 16):
            x = rng.integers(-32768, 32768, (n, 2)).astype(np.int16)
            assert (Z.v_shift_right_complex16(x, sh) == oracle.v_shift_right_complex16(x, sh)).all()


# ------------------------------------------------------------------ Viterbi
def test_viterbi_kat(golden):
    k = golden["ref_kats"]
    Z.viterbi_brick_init_fast(100, 0, 256)
    outs = []
    s = k["vit_kat_soft"]
    for i in range(0, s.size, 48):
        nb, b = Z.viterbi_brick_decode_fast(s[i:i + 48])
        outs.append(b)
    bits = np.unpackbits(np.concatenate(outs), bitorder="little")
    assert (bits == k["vit_kat_bits"]).all()


def test_viterbi_per_call_reference_frames(golden):
    """Every reference-brick frame (3 rates x lengths 1..4095 x noise levels), 48 soft values
    per call as Viterbi.blk feeds them."""
    g = golden["ref_viterbi"]
    cases, so, oo = g["vit_cases"], g["vit_soft_off"], g["vit_out_off"]
    for i, (cr, fl, noise) in enumerate(cases):
        Z.viterbi_brick_init_fast(int(fl), int(cr), 256)
        s = g["vit_soft"][so[i]:so[i + 1]]
        outs = []
        for k in range(0, s.size, 48):
            nb, b = Z.viterbi_brick_decode_fast(s[k:k + 48])
            assert nb == 8 * b.size
            outs.append(b)
        got = np.concatenate(outs)
        exp = g["vit_out"][oo[i]:oo[i + 1]]
        assert got.size >= exp.size and (got[:exp.size] == exp).all(), f"case {(cr, fl, noise)}"


def test_viterbi_adversarial_wrap_per_call(golden):
    g = golden["ref_viterbi"]
    s = g["vit_adv_soft"]
    for cr in (0, 1, 2):
        Z.viterbi_brick_init_fast(1000, cr, 256)
        outs = [Z.viterbi_brick_decode_fast(s[k:k + 48])[1] for k in range(0, s.size - 47, 48)]
        got = np.concatenate(outs)
        exp = g[f"vit_adv_out_{cr}"]
        assert (got[:exp.size] == exp).all(), cr


def test_viterbi_per_call_depths_vs_oracle(oracle):
    """Depths other than 256 and call sizes other than 48, call by call against the oracle
    (itself pinned on these cases by test_oracle_vs_ref.py)."""
    from tests.golden import synth
    from tests.test_oracle_vs_ref import _per_call_cases
    for cr, fl, noise, depth, call, seed in _per_call_cases():
        s = synth.viterbi_soft(cr, fl, noise, seed=seed)
        Z.viterbi_brick_init_fast(fl, cr, depth)
        d = oracle.Viterbi()
        d.init(fl, cr, depth)
        for k in range(0, s.size, call):
            c = np.ascontiguousarray(s[k:k + call])
            if c.size % 12:
                break
            nb, got = Z.viterbi_brick_decode_fast(c)
            exp = d.decode(c)
            assert nb == 8 * exp.size and (got == exp).all(), (cr, fl, depth, call, k)


def test_viterbi_per_call_deep_windows_vs_oracle(oracle):
    from tests.golden import synth
    for cr, depth, call in ((0, 4060, 480), (2, 4070, 96), (0, 5000, 480), (1, 8000, 4800)):
        s = synth.viterbi_soft(cr, 2000, 3, seed=depth)
        Z.viterbi_brick_init_fast(2000, cr, depth)
        d = oracle.Viterbi()
        d.init(2000, cr, depth)
        total = 0
        for k in range(0, s.size - call + 1, call):
            c = np.ascontiguousarray(s[k:k + call])
            nb, got = Z.viterbi_brick_decode_fast(c)
            exp = d.decode(c)
            assert nb == 8 * exp.size and (got == exp).all(), (cr, depth, call, k)
            total += exp.size
        assert total >= depth // 8, (cr, depth, total)


def test_viterbi_per_call_out_of_range_soft_vs_oracle(oracle):
    """Soft bytes outside 0..7 (the brick indexes its LUTs with them; both engines use the
    LUTs' closed form e ? 14 - 2v : 2v in u8 arithmetic)."""
    rng = np.random.default_rng(3)
    for cr in (0, 1, 2):
        s = rng.integers(-128, 128, 48 * 60).astype(np.int8)
        Z.viterbi_brick_init_fast(300, cr, 256)
        d = oracle.Viterbi()
        d.init(300, cr, 256)
        for k in range(0, s.size, 48):
            c = np.ascontiguousarray(s[k:k + 48])
            nb, got = Z.viterbi_brick_decode_fast(c)
            exp = d.decode(c)
            assert nb == 8 * exp.size and (got == exp).all(), (cr, k)


def test_viterbi_per_call_partial_group_and_bad_rate():
    """A partial trailing group is not consumed; an unknown code rate decodes nothing (the
    reference loops forever on it)."""
    Z.viterbi_brick_init_fast(10, 2, 256)
    nb, _ = Z.viterbi_brick_decode_fast(np.zeros(47, np.int8))
    assert nb == 0
    Z.viterbi_brick_init_fast(10, 7, 256)
    nb, _ = Z.viterbi_brick_decode_fast(np.full(480, 7, np.int8))
    assert nb == 0


def test_viterbi_per_call_trellis_cap(oracle):
    """Beyond TRELLIS_MAX = 40000 columns (sora_ext_viterbi.cpp:39) groups are not consumed
    instead of overflowing the trellis buffer; the frame's earlier windows still come out,
    equal to the oracle's (which stops at the same column)."""
    rng = np.random.default_rng(4)
    s = rng.integers(0, 8, 96000).astype(np.int8)
    Z.viterbi_brick_init_fast(6000, 0, 256)
    d = oracle.Viterbi()
    d.init(6000, 0, 256)
    total = 0
    for k in range(0, s.size, 4800):
        c = np.ascontiguousarray(s[k:k + 4800])
        nb, b = Z.viterbi_brick_decode_fast(c)
        exp = d.decode(c)
        assert nb == 8 * exp.size and (b == exp).all(), k
        total += nb
    assert 0 < total < 40000 and total % 256 == 0


# ------------------------------------------------------------------ SIGNAL
def test_signal_kat(golden):
    k = golden["ref_kats"]
    w = Z.viterbiSig11a_brick_decode_fast(k["sig_kat_soft"])
    bits = np.unpackbits(w, bitorder="little")[:24].copy()
    bits[18:] = 0
    assert (bits == k["sig_kat_bits"]).all()


def test_signal_reference_vectors(golden):
    g = golden["ref_viterbi"]
    for s, exp in zip(g["sig_soft"], g["sig_bits"]):
        w = Z.viterbiSig11a_brick_decode_fast(s)
        b = np.unpackbits(w, bitorder="little")[:24].copy()
        b[18:] = 0
        assert (np.packbits(b, bitorder="little") == exp).all()


def test_signal_random_vs_oracle(oracle):
    rng = np.random.default_rng(9)
    for _ in range(300):
        s = rng.integers(0, 8, 48).astype(np.int8)
        prev = rng.integers(0, 256, 4).astype(np.uint8)         # byte 3 is the caller's, shifted in
        got = Z.viterbiSig11a_brick_decode_fast(s, prev)
        exp = oracle.viterbi_sig(s)                           # (its byte 3 was 0)
        assert got[0] == exp[0] and got[1] == exp[1] and (got[2] & 3) == (exp[2] & 3)
        # *(unum32*)bit >>= 6 moves the caller's byte-3 bits 0..5 into bits 18..23
        assert got[2] >> 2 == prev[3] & 0x3F and got[3] == prev[3] >> 6
