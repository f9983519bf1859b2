"""Random cross-checks of the oracle against the reference bricks compiled from
/root/reference (oracle/_ref).  Skipped where those bricks are not built (GPU box)."""
import ctypes as C

import numpy as np
import pytest

from tests.golden import synth


@pytest.fixture(scope="module")
def ref(oracle):
    r = oracle.ref()
    if r is None:
        pytest.skip("reference bricks not built here (needs /root/reference)")
    return r


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def test_fft_random(oracle, ref):
    rng = np.random.default_rng(123)
    for t in range(300):
        x = rng.integers(-32768, 32768, (64, 2)).astype(np.int16)
        o = np.zeros_like(x)
        ref.zref_sora_fft(_p(o), 64, _p(x))
        assert (oracle.fft64(x) == o).all()


def test_fft_all_sizes_random(oracle, ref):
    """Every __ext_sora_fft size (csrc/sora_ext_lib.cpp:2672-2812), and a rejected size that
    leaves the output untouched."""
    rng = np.random.default_rng(321)
    for n in oracle.FFT_SIZES:
        for t in range(12):
            x = rng.integers(-32768, 32768, (n, 2)).astype(np.int16)
            if t % 3 == 1:
                x = rng.choice(np.array([-32768, 32767, -1, 0, 1], np.int16), (n, 2))
            o = np.zeros_like(x)
            ref.zref_sora_fft(_p(o), n, _p(x))
            assert (oracle.fft_n(n, x) == o).all(), (n, t)


def test_viterbi_luts(oracle, ref):
    ma = np.zeros(1024, np.uint8)
    mb = np.zeros(1024, np.uint8)
    ref.zref_viterbi_luts(_p(ma), _p(mb))
    ma, mb = ma.reshape(64, 16), mb.reshape(64, 16)
    for soft in range(8):
        for k in range(8):
            for j in range(16):
                assert ma[soft * 8 + k, j] == oracle.vit_lut(0, soft, k, j)
                assert mb[soft * 8 + k, j] == oracle.vit_lut(1, soft, k, j)


def test_viterbi_random(oracle, ref):
    rng = np.random.default_rng(9)
    buf = np.zeros(12000, np.uint8)
    for i in range(24):
        cr, fl = int(rng.integers(0, 3)), int(rng.integers(1, 400))
        s = synth.viterbi_soft(cr, fl, int(rng.integers(-1, 6)), seed=77 + i)
        ref.zref_viterbi_init(fl, cr, 256)
        outs = []
        for k in range(0, s.size, 48):
            c = np.ascontiguousarray(s[k:k + 48])
            bits = ref.zref_viterbi_decode(_p(c), 48, _p(buf), 96000)
            outs.append(buf[:bits // 8].copy())
        assert (np.concatenate(outs) == oracle.viterbi_decode(s, fl, cr)).all()


def _per_call_cases():
    """(code rate, frame length, noise, depth, call size) for the per-call path: depths other
    than the WiFi RX's 256 (the brick honours any, sora_ext_viterbi.cpp:55-56) and call
    sizes other than 48 (whole groups of every rate: multiples of 12)."""
    rng = np.random.default_rng(0xDE)
    out = []
    for i, depth in enumerate((32, 64, 100, 200, 256, 300, 512, 1000)):
        for cr in (0, 1, 2):
            out.append((cr, int(rng.integers(1, 700)), int(rng.integers(-1, 6)), depth,
                        int(rng.choice([12, 24, 48, 96, 480])), 500 + 10 * i + cr))
    return out


def test_viterbi_depths_and_call_sizes(oracle, ref):
    buf = np.zeros(96000, np.uint8)
    for cr, fl, noise, depth, call, seed in _per_call_cases():
        s = synth.viterbi_soft(cr, fl, noise, seed=seed)
        ref.zref_viterbi_init(fl, cr, depth)
        d = oracle.Viterbi()
        d.init(fl, cr, depth)
        for k in range(0, s.size, call):
            c = np.ascontiguousarray(s[k:k + call])
            if c.size % 12:
                break
            bits = ref.zref_viterbi_decode(_p(c), c.size, _p(buf), buf.size * 8)
            got = d.decode(c)
            assert got.size * 8 == bits and (got == buf[:bits // 8]).all(), (cr, fl, depth, call, k)


def test_shift_right(oracle, ref):
    rng = np.random.default_rng(5)
    for n in (1, 3, 4, 5, 9):
        for sh in (0, 1, 15, 16, 20):
            x = rng.integers(-32768, 32768, (n, 2)).astype(np.int16)
            z = np.zeros_like(x)
            ref.zref_v_shift_right_complex16(_p(z), _p(x), n, sh)
            assert (z == oracle.v_shift_right_complex16(x, sh)).all()


def test_trig_exhaustive(oracle, ref):
    L = oracle.lib()
    s, c, _ = oracle.trig_tables()
    r = np.arange(65536).astype(np.uint16).astype(np.int16)
    rs = np.array([ref.zref_sin16(int(v)) for v in r], np.int16)
    rc = np.array([ref.zref_cos16(int(v)) for v in r], np.int16)
    assert (s == rs).all() and (c == rc).all()
    g = np.arange(-300, 301)
    for y in g[::7]:
        for x in g:
            assert oracle.atan2_16(y, x) == ref.zref_atan2_16(int(y), int(x)), (y, x)
    rng = np.random.default_rng(31)
    for y, x in rng.integers(-32768, 32768, (5000, 2)):
        assert oracle.atan2_16(y, x) == ref.zref_atan2_16(int(y), int(x)), (y, x)


def test_v_mul_complex16(oracle, ref):
    rng = np.random.default_rng(8)
    for n in (1, 3, 4, 7, 28, 64):
        for sh in (0, 8, 15, 16):
            x = rng.integers(-32768, 32768, (n, 2)).astype(np.int16)
            y = rng.integers(-32768, 32768, (n, 2)).astype(np.int16)
            x[0] = y[0] = (-32768, -32768)
            z = np.zeros_like(x)
            ref.zref_v_mul_complex16(_p(z), _p(x), _p(y), n, sh)
            assert (z == oracle.v_mul_complex16(x, y, sh)).all(), (n, sh)
