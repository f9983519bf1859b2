"""GPU parity of k_viterbi3's trellis segments (zrx_viterbi3.hpp "Trellis segments"): batches
too small to fill the GPU are decoded as segments of their frames, seams checked, disagreeing
seams re-decoded by the fix pass.  Every comparison is bit-exact against the oracle's unsplit
decode (or the transmitted bits), and the plan statistics show which path ran."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from ziria_amd.engine import RxEngine  # noqa: E402
from tests.golden import synth  # noqa: E402


def _run(frames, reserve=None):
    """frames: list of (soft int8, frame_len, code_rate) -> (out bytes per frame, out_bits,
    plan stats) through zrx_viterbi_dev."""
    n = len(frames)
    sl = np.array([f[0].size for f in frames], np.int64)
    so = np.cumsum(sl) - sl
    fl = np.array([f[1] for f in frames], np.int64)
    oo = np.cumsum(fl + 16) - (fl + 16)
    soft = torch.from_numpy(np.concatenate([f[0] for f in frames])).cuda()
    params = torch.from_numpy(np.stack([fl, [f[2] for f in frames], sl, np.zeros(n)], 1).astype(np.int32)).cuda()
    out = torch.zeros(int(oo[-1] + fl[-1] + 16), dtype=torch.uint8, device="cuda")
    ob = torch.zeros(n, dtype=torch.int32, device="cuda")
    e = RxEngine(0)
    e.reserve(reserve or n, 1)
    e.viterbi(soft, torch.from_numpy(so).cuda(), params.contiguous(), out, torch.from_numpy(oo).cuda(), ob)
    torch.cuda.synchronize()
    st = e.plan_stats()
    e.close()
    o = out.cpu().numpy()
    return [o[oo[i]:oo[i] + fl[i]] for i in range(n)], ob.cpu().numpy(), st


def test_segments_all_rates_and_noise_vs_oracle(oracle):
    """48 long frames (1500..4095 B, all rates, clean to pure noise): a batch this small is cut
    into up to 8 segments per frame; pure-noise frames make seams disagree, so the fix pass
    runs too.  Every byte and bit count equals the oracle's."""
    rng = np.random.default_rng(2024)
    frames = []
    for i in range(48):
        cr = i % 3
        fl = int(rng.integers(1500, 4096))
        noise = (-1, 0, 2, 3, 4, -1)[i % 6]
        frames.append((synth.viterbi_soft(cr, fl, noise, seed=7000 + i), fl, cr))
    got, bits, (rows, fixes) = _run(frames)
    assert rows > 6 * len(frames)                        # long frames were cut
    assert fixes > 0                                     # some pure-noise seam disagreed
    for i, (s, fl, cr) in enumerate(frames):
        exp = oracle.viterbi_decode(s, fl, cr)
        assert bits[i] == 8 * exp.size, i
        assert (got[i] == exp).all(), i


def test_segments_config2_shape():
    """BASELINE config 2 (4096 x 1500 B, R=1/2, soft 7*bit + U[-2,2]): four segments per frame
    (16384 rows), no seam disagrees, every frame equals the transmitted bits."""
    from ziria_amd import txgen
    n, fl = 4096, 1500
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED)
    L = -(-(8 * fl + 6) // 24) * 24
    u = torch.zeros((n, L), dtype=torch.uint8, device="cuda")
    u[:, :8 * fl] = torch.randint(0, 2, (n, 8 * fl), generator=g, device="cuda", dtype=torch.uint8)
    coded = txgen._encode(u, 0).to(torch.int16)
    soft = torch.clamp(coded * 7 + torch.randint(-2, 3, coded.shape, generator=g, device="cuda",
                                                 dtype=torch.int16), 0, 7).to(torch.int8).contiguous()
    ns = soft.shape[1]
    params = torch.tensor([fl, 0, ns, 0], dtype=torch.int32, device="cuda").repeat(n, 1).contiguous()
    out = torch.zeros(n * 1504, dtype=torch.uint8, device="cuda")
    ob = torch.zeros(n, dtype=torch.int32, device="cuda")
    e = RxEngine(0)
    e.reserve(n, 1)
    e.viterbi(soft.reshape(-1), torch.arange(n, device="cuda", dtype=torch.int64) * ns, params, out,
              torch.arange(n, device="cuda", dtype=torch.int64) * 1504, ob)
    torch.cuda.synchronize()
    rows, fixes = e.plan_stats()
    e.close()
    assert rows == 4 * n and fixes == 0
    sent = np.packbits(u[:, :8 * fl].cpu().numpy(), axis=1, bitorder="little")
    assert (out.reshape(n, 1504)[:, :fl].cpu().numpy() == sent).all()
    assert (ob.cpu().numpy() == 8 * fl).all()


def test_segments_not_cut_when_gpu_full():
    """16384 equal 54 Mbps-length frames fill every SIMD with four waves: one row per frame."""
    fl, cr = 1506, 2
    s = synth.viterbi_soft(cr, fl, 2, seed=5)
    frames = [(s, fl, cr)] * 16384
    got, bits, (rows, fixes) = _run(frames)
    assert rows == 16384 and fixes == 0
    assert all((g == got[0]).all() for g in got[::257])
    assert (bits == 8 * fl).all()


def test_segments_mixed_lengths_and_truncation(oracle):
    """Short, long and truncated frames in one small batch: long complete frames are cut,
    truncated ones (input ends mid-frame) and short ones are not; all equal the oracle."""
    rng = np.random.default_rng(99)
    frames = []
    for i in range(40):
        cr = int(rng.integers(0, 3))
        fl = int(rng.choice([5, 60, 400, 2048, 4095]))
        s = synth.viterbi_soft(cr, fl, int(rng.integers(0, 4)), seed=900 + i)
        if i % 4 == 3:
            s = s[: max(48, (s.size * 2 // 3) // 48 * 48)]
        frames.append((s, fl, cr))
    got, bits, (rows, _) = _run(frames)
    assert rows > len(frames)
    for i, (s, fl, cr) in enumerate(frames):
        exp = oracle.viterbi_decode(s, fl, cr)
        assert bits[i] == 8 * exp.size, i
        assert (got[i][:exp.size] == exp).all(), i


def test_segments_uniform_batch_with_fixes(oracle):
    """64 frames with equal parameters (a uniform batch: rows derived in k_viterbi3, no row
    table) but pure-noise soft values: cut into segments, some seams disagree and the seam pass
    re-decodes them; every frame equals the oracle."""
    fl, cr = 3000, 2
    frames = [(synth.viterbi_soft(cr, fl, -1, seed=3000 + i), fl, cr) for i in range(64)]
    got, bits, (rows, fixes) = _run(frames)
    assert rows == 64 * 8 and fixes > 0
    for i, (s, _, _) in enumerate(frames):
        exp = oracle.viterbi_decode(s, fl, cr)
        assert bits[i] == 8 * fl and (got[i] == exp).all(), i


def test_segments_small_uniform_batch_min_cut(oracle):
    """A small uniform batch is cut down to kMinCut-column segments (v3::seg_count with
    kMinCut): 600-byte frames (E = 4806) take 4 segments starting at units 0, 2, 3, 5, so one
    segment spans a single 768-column unit.  Half the frames are pure noise (seams disagree,
    the fix pass runs); every frame equals the oracle."""
    fl, cr = 600, 1
    frames = [(synth.viterbi_soft(cr, fl, -1 if i % 2 else 2, seed=4100 + i), fl, cr) for i in range(128)]
    got, bits, (rows, fixes) = _run(frames)
    assert rows == 128 * 4 and fixes > 0
    for i, (s, _, _) in enumerate(frames):
        exp = oracle.viterbi_decode(s, fl, cr)
        assert bits[i] == 8 * fl and (got[i] == exp).all(), i


def test_segments_config4_shard(oracle):
    """The per-GPU Viterbi of config 4 at N = 8 (2048 frames of 1504 B at rate 3/4, a config-3
    shard): 8 segments per frame, i.e. 16384 rows (two waves per SIMD); 16 distinct frames
    tiled, each equal to the oracle."""
    fl, cr = 1504, 2
    base = [(synth.viterbi_soft(cr, fl, 3, seed=4300 + i), fl, cr) for i in range(16)]
    got, bits, (rows, fixes) = _run(base * 128)
    assert rows == 2048 * 8 and fixes == 0
    exp = [oracle.viterbi_decode(s, fl, cr) for s, _, _ in base]
    assert (bits == 8 * fl).all()
    for i, g in enumerate(got):
        assert (g == exp[i % 16]).all(), i
