"""GPU parity: the HIP engine (through the C-ABI of libziria_rx.so) against the oracle, the
reference's own KATs and the reference-brick golden fixtures.  Integer/byte work, so every
comparison is bit-exact (no tolerance).  The per-call externals run on the host and are
tested without a GPU in tests/test_percall_host.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import ziria_amd as Z  # noqa: E402
from ziria_amd import txgen  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402


@pytest.fixture(scope="module")
def engine():
    e = RxEngine(0)
    yield e
    e.close()


def test_library_is_native():
    assert Z.lib().zrx_version().startswith(b"ziria_rx")


# ------------------------------------------------------------------ FFT64
def test_fft64_reference_vectors(golden):
    g = golden["ref_fft64"]
    out = Z.sora_fft64_batch(g["fft_in"])
    assert (out == g["fft_out"]).all()


def test_fft64_device_random_vs_oracle(engine, oracle):
    rng = np.random.default_rng(11)
    x = rng.integers(-32768, 32768, (3000, 64, 2)).astype(np.int16)
    x[:500] = rng.choice(np.array([-32768, 32767, -1, 0], np.int16), (500, 64, 2))
    out = engine.fft64(torch.from_numpy(x).cuda()).cpu().numpy()
    assert (out == oracle.fft64(x)).all()


def test_fft_all_sizes_reference_vectors(engine, golden):
    """zrx_fft_dev on the reference brick's outputs for random, saturating and small vectors
    of every size (one batch per size)."""
    g = golden["ref_fftn"]
    o, per = g["vec_off"], int(g["vec_per"])
    for i, n in enumerate(g["sizes"]):
        n = int(n)
        a, b = o[i * per], o[(i + 1) * per]
        x = torch.from_numpy(np.ascontiguousarray(g["vec_in"][a:b].reshape(per, n, 2))).cuda()
        assert (engine.fft(n, x).cpu().numpy().reshape(-1, 2) == g["vec_out"][a:b]).all(), n


def test_fft_all_sizes_random_vs_oracle(engine, oracle):
    """Batches past the kernel's grid (block-stride loop) and in-place transforms."""
    rng = np.random.default_rng(42)
    for n in oracle.FFT_SIZES:
        cnt = 3000 if n <= 16 else 40
        x = rng.integers(-32768, 32768, (cnt, n, 2)).astype(np.int16)
        x[: cnt // 4] = rng.choice(np.array([-32768, 32767, -1, 0, 1], np.int16), (cnt // 4, n, 2))
        exp = oracle.fft_n(n, x)
        d = torch.from_numpy(x).cuda()
        assert (engine.fft(n, d).cpu().numpy() == exp).all(), n
        engine.fft(n, d, out=d)                              # aliasing in/out
        assert (d.cpu().numpy() == exp).all(), n


# ------------------------------------------------------------------ Viterbi
def _vit_cases(golden):
    g = golden["ref_viterbi"]
    return g, g["vit_cases"], g["vit_soft_off"], g["vit_out_off"]


def test_viterbi_batch_reference_frames(golden):
    g, cases, so, oo = _vit_cases(golden)
    fl = cases[:, 1].astype(np.int32)
    cr = cases[:, 0].astype(np.int16)
    out, off = Z.viterbi_batch_decode(g["vit_soft"], so.astype(np.int32), fl, cr)
    for i in range(len(cases)):
        exp = g["vit_out"][oo[i]:oo[i + 1]]
        got = out[off[i]:off[i] + exp.size]
        assert (got == exp).all(), f"case {tuple(cases[i])}"


def test_viterbi_adversarial_wrap(golden):
    g = golden["ref_viterbi"]
    s = g["vit_adv_soft"]
    for cr in (0, 1, 2):
        out, _ = Z.viterbi_batch_decode(s, np.array([0, s.size], np.int32), np.array([1000], np.int32),
                                        np.array([cr], np.int16))
        exp = g[f"vit_adv_out_{cr}"]
        assert (out[:exp.size] == exp).all()


def test_viterbi_batch_random_vs_oracle(oracle):
    rng = np.random.default_rng(77)
    softs, offs, fls, crs = [], [0], [], []
    for i in range(67):                          # not a multiple of 4 packets per block
        cr = int(rng.integers(0, 3))
        fl = int(rng.integers(1, 700))
        from tests.golden import synth
        s = synth.viterbi_soft(cr, fl, int(rng.integers(-1, 5)), seed=1000 + i)
        if i % 5 == 0:
            s = s[: max(48, (s.size // 2) // 48 * 48)]      # truncated: decoder stops mid-frame
        softs.append(s); offs.append(offs[-1] + s.size); fls.append(fl); crs.append(cr)
    soft = np.concatenate(softs)
    out, off = Z.viterbi_batch_decode(soft, np.array(offs, np.int32), np.array(fls, np.int32),
                                      np.array(crs, np.int16))
    for i in range(len(fls)):
        exp = oracle.viterbi_decode(soft[offs[i]:offs[i + 1]], fls[i], crs[i])
        assert (out[off[i]:off[i] + exp.size] == exp).all(), i


def test_viterbi_empty_batch():
    out, off = Z.viterbi_batch_decode(np.zeros(0, np.int8), np.array([0], np.int32),
                                      np.zeros(0, np.int32), np.zeros(0, np.int16))
    assert off.size == 0


# ------------------------------------------------------------------ full chain
def _check_chain(pay, info, exp_pay, exp_off, exp_crc, meta):
    for i in range(len(exp_crc)):
        mod, cod, ln = meta[i]
        assert info["modulation"][i] == mod and info["coding"][i] == cod and info["len"][i] == ln
        assert info["crc_ok"][i] == exp_crc[i], i
        e = exp_pay[exp_off[i]:exp_off[i + 1]]
        assert (pay[i, :e.size] == e).all(), i


@pytest.mark.parametrize("tag", ["c54", "mix"])
def test_chain_reference_packets(golden, tag):
    g = golden["ref_chain"]
    sym, off, nsym = g[f"{tag}_sym"], g[f"{tag}_off"], g[f"{tag}_nsym"]
    csr = np.concatenate([off, [off[-1] + nsym[-1]]]).astype(np.int32)
    pay, info, nok = Z.wifi_rx_batch(sym, csr)
    _check_chain(pay, info, g[f"{tag}_payload"], g[f"{tag}_payload_off"], g[f"{tag}_crc"], g[f"{tag}_meta"])
    assert nok == int(g[f"{tag}_crc"].sum())


def test_chain_device_engine_54mbps(engine, oracle):
    b = txgen.make_batch(257, seed=99, device="cuda")
    engine.reserve(257, b["max_nsym"])
    pay, info = engine.rx(b["sym"], b["sym_off"], b["nsym"], b["max_nsym"])
    pay, info = pay.cpu().numpy(), info.cpu().numpy()
    assert (info[:, 4] == 1).all() and (info[:, 5] == 0).all()
    assert (pay[:, :1500] == b["payload"]).all()
    opay, ores = oracle.rx_batch_time(b["sym"].cpu().numpy(), b["sym_off"].cpu().numpy(),
                                      b["nsym"].cpu().numpy(), nthreads=8)
    assert (pay[:, :1500] == opay[:, :1500]).all()
    assert all(r["crc_ok"] == 1 for r in ores)


@pytest.mark.parametrize("mod,coding", [(0, 0), (0, 2), (1, 0), (1, 2), (2, 0), (2, 2), (3, 1), (3, 2)])
def test_chain_uniform_mcs_vs_oracle(engine, oracle, mod, coding):
    """Every 802.11a rate alone: waves of one modulation, so k_data_fft's store loop runs the
    3 / 6 / 12 / 18 iterations of that soft row (the mixed tests run the widest of a wave)."""
    b = txgen.make_batch(130, mod=mod, coding=coding, payload_len=211, sigma=2.0, seed=0x3C + 8 * mod + coding,
                         device="cuda")
    engine.reserve(130, b["max_nsym"])
    pay, info = engine.rx(b["sym"], b["sym_off"], b["nsym"], b["max_nsym"])
    pay, info = pay.cpu().numpy(), info.cpu().numpy()
    assert (info[:, 0] == mod).all() and (info[:, 1] == coding).all() and (info[:, 4] == 1).all()
    assert (pay[:, :211] == b["payload"]).all()
    opay, ores = oracle.rx_batch_time(b["sym"].cpu().numpy(), b["sym_off"].cpu().numpy(),
                                      b["nsym"].cpu().numpy(), nthreads=8)
    assert all(r["crc_ok"] == 1 for r in ores)
    assert (pay[:, :211] == opay[:, :211]).all()


def test_chain_mixed_mcs_vs_oracle(engine, oracle):
    m = txgen.make_mixed(96, max_len=2200, sigma=3.0, seed=5, device="cuda")
    n = m["sym_off"].numel()
    engine.reserve(n, m["max_nsym"])
    pay, info = engine.rx(m["sym"], m["sym_off"], m["nsym"], m["max_nsym"])
    pay, info = pay.cpu().numpy(), info.cpu().numpy()
    opay, ores = oracle.rx_batch_time(m["sym"].cpu().numpy(), m["sym_off"].cpu().numpy(),
                                      m["nsym"].cpu().numpy(), nthreads=8)
    for i in range(n):
        r = ores[i]
        assert (info[i, 0], info[i, 1], info[i, 2], info[i, 3]) == (r["modulation"], r["coding"], r["len"], r["err"])
        if r["err"]:
            assert info[i, 5] == 1 and info[i, 4] == 0
            continue
        assert info[i, 4] == r["crc_ok"]
        L = r["len"] - 4
        assert (pay[i, :L] == opay[i, :L]).all(), i
    ok = info[:, 3] == 0
    assert ok.sum() > 40 and (info[ok, 4] == 1).all()


def test_chain_truncated_and_bad_header(engine, oracle):
    b = txgen.make_batch(8, seed=4, device="cuda")
    sym = b["sym"].clone()
    nsym = b["nsym"].clone()
    nsym[1] = 10                                # fewer symbols than the header needs
    S = b["max_nsym"]
    sym[2 * S] = 0                              # zeroed SIGNAL symbol -> header garbage
    engine.reserve(8, S)
    pay, info = engine.rx(sym, b["sym_off"], nsym, S)
    info = info.cpu().numpy()
    assert info[1, 5] == 2 and info[1, 4] == 0
    _, r2 = oracle.rx_packet_time(sym[2 * S:3 * S].cpu().numpy())
    assert (info[2, 0], info[2, 1], info[2, 2], info[2, 3]) == (r2["modulation"], r2["coding"], r2["len"], r2["err"])
    for i in (0, 3, 4, 5, 6, 7):
        assert info[i, 4] == 1


def test_chain_mixed_distinct_large(engine, oracle):
    """BASELINE config 5 shape at 2048 distinct packets (PSDU 64..4095 B, all 8 MCS, long
    6 Mbps packets): every packet with a valid header passes its CRC with the transmitted
    payload, and a sample equals the oracle packet for packet (mixed rates and lengths in a
    wave, ordered rows, packed soft slots, shared and per-row traceback windows)."""
    m = txgen.make_mixed_fast(2048, min_len=64, max_len=4095, sigma=3.0, seed=0xC5C5, device="cuda")
    n = m["sym_off"].numel()
    engine.reserve(n, m["max_nsym"])
    pay, info = engine.rx(m["sym"], m["sym_off"], m["nsym"], m["max_nsym"])
    engine.plan_check()                                   # no Viterbi row dropped past the plan's bound
    pay, info = pay.cpu().numpy(), info.cpu().numpy()
    valid = m["meta"][:, 2] <= 2048
    assert (info[valid, 4] == 1).all(), np.nonzero(valid & (info[:, 4] != 1))[0][:10]
    assert (info[~valid, 3] == 1).all()
    for i in np.nonzero(valid)[0]:
        assert (pay[i, :m["meta"][i, 2] - 4] == m["payload"][i]).all(), i
    sample = 96
    soff, sn = m["sym_off"][:sample].cpu().numpy(), m["nsym"][:sample].cpu().numpy()
    opay, res = oracle.rx_batch_time(m["sym"][:int((soff + sn).max())].cpu().numpy(), soff, sn, nthreads=8)
    for i, r in enumerate(res):
        assert (info[i, 2], info[i, 4]) == (r["len"], r["crc_ok"]), i
        if r["crc_ok"]:
            assert (pay[i, :r["len"] - 4] == opay[i, :r["len"] - 4]).all(), i


def test_viterbi_order_large_mixed_batch(oracle):
    """k_vit_order past the old 32768-packet LDS cap: 40000 frames of mixed rates and
    lengths (1..60 bytes, plus a few of 2048) through the device API equal the oracle."""
    rng = np.random.default_rng(40000)
    n = 40000
    fl = rng.integers(1, 61, n).astype(np.int32)
    fl[rng.choice(n, 8, replace=False)] = 2048
    cr = rng.integers(0, 3, n).astype(np.int16)
    K = np.array([24, 32, 36])[cr]
    sl = ((8 * fl + 6 + K - 1) // K * 48).astype(np.int32)
    so = (np.cumsum(sl) - sl).astype(np.int64)
    soft = rng.integers(0, 8, int(sl.sum())).astype(np.int8)
    oo = (np.cumsum(fl + 8) - (fl + 8)).astype(np.int64)
    exp = oracle.viterbi_batch(soft, so, sl, fl, cr, oo, int(oo[-1] + fl[-1] + 8), nthreads=8)
    params = torch.from_numpy(np.stack([fl, cr.astype(np.int32), sl, np.zeros(n, np.int32)], 1).copy()).cuda()
    out = torch.zeros(int(oo[-1] + fl[-1] + 8), dtype=torch.uint8, device="cuda")
    ob = torch.zeros(n, dtype=torch.int32, device="cuda")
    e = RxEngine(0)
    e.reserve(n, 1)                                      # room for the packet order
    e.viterbi(torch.from_numpy(soft).cuda(), torch.from_numpy(so).cuda(), params, out,
              torch.from_numpy(oo).cuda(), ob)
    torch.cuda.synchronize()
    e.close()
    got = out.cpu().numpy()
    assert (ob.cpu().numpy() == 8 * fl).all()
    for i in range(n):
        assert (got[oo[i]:oo[i] + fl[i]] == exp[oo[i]:oo[i] + fl[i]]).all(), i


def test_chain_mixed_order_rounds_and_partial_block(engine, oracle):
    """4100 mixed packets: k_pkt_plan's packet order spans more than one round of CU blocks
    (snake placement reverses the second) and ends in a partial block of 4 rows; every packet
    with a valid header decodes to its payload, and a sample equals the oracle."""
    m = txgen.make_mixed_fast(4100, min_len=64, max_len=700, sigma=3.0, seed=4100, device="cuda")
    n = m["sym_off"].numel()
    engine.reserve(n, m["max_nsym"])
    pay, info = engine.rx(m["sym"], m["sym_off"], m["nsym"], m["max_nsym"])
    pay, info = pay.cpu().numpy(), info.cpu().numpy()
    assert (info[:, 4] == 1).all()
    for i in range(n):
        assert (pay[i, :m["meta"][i, 2] - 4] == m["payload"][i]).all(), i
    sample = np.arange(n - 64, n)                          # the partial block and its neighbours
    soff, sn = m["sym_off"].cpu().numpy(), m["nsym"].cpu().numpy()
    sym = m["sym"].cpu().numpy()
    opay, res = oracle.rx_batch_time(sym, soff[sample], sn[sample], nthreads=8)
    for j, r in enumerate(res):
        i = sample[j]
        assert (info[i, 2], info[i, 4]) == (r["len"], r["crc_ok"]), i
        assert (pay[i, :r["len"] - 4] == opay[j, :r["len"] - 4]).all(), i


def test_viterbi_soft_spread_beyond_window():
    """Rows of a wave whose soft values lie more than 4 GiB apart (device API) decode one at a
    time, exactly."""
    if torch.cuda.get_device_properties(0).total_memory < 12 << 30:
        pytest.skip("needs > 12 GiB")
    from tests.golden import synth
    fl, cr = 300, 2
    s = synth.viterbi_soft(cr, fl, 3, seed=41)
    gap = (5 << 30) // 256 * 256
    big = torch.zeros(gap + s.size + 4096, dtype=torch.int8, device="cuda")
    srcs = torch.from_numpy(s).cuda()
    big[:s.size] = srcs
    big[gap:gap + s.size] = srcs
    off = torch.tensor([0, gap, 0, gap], dtype=torch.int64, device="cuda")
    params = torch.tensor([fl, cr, s.size, 0], dtype=torch.int32, device="cuda").repeat(4, 1).contiguous()
    out = torch.zeros(4 * 512, dtype=torch.uint8, device="cuda")
    oo = torch.arange(4, dtype=torch.int64, device="cuda") * 512
    ob = torch.zeros(4, dtype=torch.int32, device="cuda")
    e = RxEngine(0)
    e.viterbi(big, off, params, out, oo, ob)
    torch.cuda.synchronize()
    e.close()
    del big
    exp = Z.viterbi_batch_decode(s, np.array([0, s.size], np.int32), np.array([fl], np.int32), np.array([cr], np.int16))[0][:fl]
    o = out.cpu().numpy().reshape(4, 512)
    assert (ob.cpu().numpy() == 8 * fl).all()
    assert (o[:, :fl] == exp).all()


def test_chain_nsym_beyond_reservation():
    """d_nsym larger than the reserved workspace: packets whose header needs more
    symbols than a soft slot holds get ZRX_PKT_OVERSIZE and nothing is written past their
    slot; the short packets around them still decode exactly."""
    short = txgen.make_batch(3, payload_len=100, seed=21, device="cuda")       # 5 symbols each
    long = txgen.make_batch(2, payload_len=1500, seed=22, device="cuda")       # 57 symbols each
    Ss, Sl = short["max_nsym"], long["max_nsym"]
    sym = torch.cat([short["sym"][:Ss], long["sym"][:Sl], short["sym"][Ss:2 * Ss], long["sym"][Sl:],
                     short["sym"][2 * Ss:]])
    nsym = torch.tensor([Ss, Sl, Ss, Sl, Ss], dtype=torch.int32, device="cuda")
    off = torch.cumsum(torch.cat([torch.zeros(1, dtype=torch.int64, device="cuda"), nsym.to(torch.int64)]), 0)[:5]
    e = RxEngine(0)
    e.reserve(5, 12)                                     # room for 11 data symbols per packet
    pay, info = e.rx(sym.contiguous(), off.contiguous(), nsym, 12)
    pay, info = pay.cpu().numpy(), info.cpu().numpy()
    e.close()
    for i, j in ((0, 0), (2, 1), (4, 2)):
        assert info[i, 5] == 0 and info[i, 4] == 1
        assert (pay[i, :100] == short["payload"][j]).all()
    for i in (1, 3):
        assert info[i, 5] == 3 and info[i, 4] == 0 and info[i, 2] == 1504
        assert (pay[i] == 0).all()


@pytest.mark.parametrize("sigma", [55.0, 60.0])
def test_chain_54mbps_at_noise_edge_vs_oracle(engine, oracle, sigma):
    """Config-3 shape where the channel noise makes a quarter to a half of the CRCs fail
    (near-tie metrics, wrong survivors): every packet's header fields, CRC verdict and
    payload bytes (CRC-failing ones included) equal the oracle's."""
    b = txgen.make_batch(1024, seed=int(sigma), sigma=sigma, device="cuda")
    engine.reserve(1024, b["max_nsym"])
    pay, info = engine.rx(b["sym"], b["sym_off"], b["nsym"], b["max_nsym"])
    pay, info = pay.cpu().numpy(), info.cpu().numpy()
    opay, ores = oracle.rx_batch_time(b["sym"].cpu().numpy(), b["sym_off"].cpu().numpy(),
                                      b["nsym"].cpu().numpy(), nthreads=8)
    crc = np.array([r["crc_ok"] for r in ores])
    assert 100 < (crc == 0).sum() < 1000                 # the edge is really exercised
    for i, r in enumerate(ores):
        assert (info[i, 2], info[i, 3], info[i, 4]) == (r["len"], r["err"], r["crc_ok"]), i
        if not r["err"]:
            assert (pay[i, :r["len"] - 4] == opay[i, :r["len"] - 4]).all(), i


def test_chain_large_batch_properties(engine):
    """Full-size property check at config-3 shape: every CRC passes and every payload
    equals what was transmitted."""
    b = txgen.make_batch(4096, seed=1234, device="cuda")
    engine.reserve(4096, b["max_nsym"])
    pay, info = engine.rx(b["sym"], b["sym_off"], b["nsym"], b["max_nsym"])
    info = info.cpu().numpy()
    assert (info[:, 4] == 1).all()
    assert (pay[:, :1500].cpu().numpy() == b["payload"]).all()


def test_chain_split_plan_alternating_batches(engine):
    """The rx chain sorts a mixed batch's rows beside k_data_fft only when the previous batch
    was mixed (k_pkt_plan's host-mapped hint), otherwise inline: mixed and uniform batches in
    turn on one engine take both paths, from fresh and stale hints, with identical results."""
    m = txgen.make_mixed_fast(2048, min_len=64, max_len=2300, sigma=3.0, seed=77, device="cuda")
    u = txgen.make_batch(1024, seed=78, sigma=4.0, device="cuda")
    engine.reserve(2048, max(m["max_nsym"], u["max_nsym"]))
    runs = {"m": [], "u": []}
    for k in "mmumuum":
        b = m if k == "m" else u
        pay, info = engine.rx(b["sym"], b["sym_off"], b["nsym"], b["max_nsym"])
        torch.cuda.synchronize()
        runs[k].append((pay.cpu().numpy().copy(), info.cpu().numpy().copy()))
    for k, rs in runs.items():
        for pay, info in rs[1:]:
            assert (pay == rs[0][0]).all() and (info == rs[0][1]).all(), k
    pay, info = runs["m"][0]
    valid = m["meta"][:, 2] <= 2048
    assert (info[valid, 4] == 1).all()
    for i in np.nonzero(valid)[0][:512]:
        assert (pay[i, :m["meta"][i, 2] - 4] == m["payload"][i]).all(), i
    assert (runs["u"][0][1][:, 4] == 1).all()


def test_chain_plan_reuse(engine):
    """k_pkt_plan reuses the last plan when a batch is uniform and equal to the last planned
    one in size and parameters (zrx_viterbi3.hpp PlanWord; k_signal_vit raises a mismatch
    otherwise): uniform batches of one shape in turn (reused), the same size with other
    parameters (rebuilt), the same size with one truncated packet (a mismatch raised by one
    packet), a different size, and the first shape again; every batch's payloads equal what
    was sent and the plan statistics match a fresh engine's."""
    a = [txgen.make_batch(512, payload_len=1500, seed=90 + j, sigma=4.0, device="cuda") for j in range(2)]
    b = txgen.make_batch(512, payload_len=700, seed=92, sigma=4.0, device="cuda")
    c = txgen.make_batch(300, payload_len=1500, seed=93, sigma=4.0, device="cuda")
    t = txgen.make_batch(512, payload_len=1500, seed=94, sigma=4.0, device="cuda")
    nsym_t = t["nsym"].clone()
    nsym_t[200] -= 5                                   # one truncated packet: status 2, no soft values
    S = max(x["max_nsym"] for x in a + [b, c, t])
    engine.reserve(512, S)
    fresh = RxEngine(0)
    fresh.reserve(512, S)

    def check(x, nsym, pay, info, bad=()):
        pay, info = pay.cpu().numpy(), info.cpu().numpy()
        for i in range(nsym.numel()):
            if i in bad:
                assert info[i, 5] == 2 and info[i, 4] == 0, i
            else:
                assert info[i, 4] == 1 and (pay[i, :len(x["payload"][i])] == x["payload"][i]).all(), i

    # a device-API Viterbi batch of the same packet count on the same engine between two equal
    # rx batches: its plan replaces the rx plan, so the next rx batch must be planned afresh
    g = torch.Generator(device="cuda")
    g.manual_seed(95)
    ns = 12048 // 24 * 48 + 48
    vit = dict(soft=torch.randint(0, 8, (512 * ns,), generator=g, device="cuda", dtype=torch.int8),
               soft_off=torch.arange(512, dtype=torch.int64, device="cuda") * ns,
               params=torch.tensor([1000, 1, ns, 0], dtype=torch.int32, device="cuda").repeat(512, 1).contiguous(),
               out_off=torch.arange(512, dtype=torch.int64, device="cuda") * 1024)

    def run_vit(e):
        out = torch.zeros(512 * 1024, dtype=torch.uint8, device="cuda")
        bits = torch.zeros(512, dtype=torch.int32, device="cuda")
        e.viterbi(vit["soft"], vit["soft_off"], vit["params"], out, vit["out_off"], bits)
        return out, bits

    seq = [(a[0], a[0]["nsym"], ()), (a[1], a[1]["nsym"], ()), (a[0], a[0]["nsym"], ()), (b, b["nsym"], ()),
           (a[1], a[1]["nsym"], ()), (t, nsym_t, (200,)), (a[1], a[1]["nsym"], ()), (c, c["nsym"], ()),
           (a[0], a[0]["nsym"], ()), ("vit", None, ()), (a[0], a[0]["nsym"], ())]
    for x, nsym, bad in seq:
        if x == "vit":
            vo, vb = run_vit(engine)
            fo, fb = run_vit(fresh)
            torch.cuda.synchronize()
            assert (vo == fo).all() and (vb == fb).all() and (vb == 8000).all()
            continue
        pay, info = engine.rx(x["sym"], x["sym_off"], nsym, S)
        st = engine.plan_stats()
        pf, inf = fresh.rx(x["sym"], x["sym_off"], nsym, S)
        torch.cuda.synchronize()
        assert st == fresh.plan_stats()
        fresh.close()
        fresh = RxEngine(0)
        fresh.reserve(512, S)
        assert (pay == pf).all() and (info == inf).all()
        check(x, nsym, pay, info, bad)


@pytest.mark.parametrize("mode", [1, 2, 4, 5, 6, 7, 9, 13])
def test_chain_linked_engines(mode):
    """Two engines linked (zrx_pipeline_link bits: 1 the Viterbi waits for the peer's chain,
    2 the data FFT waits for the peer's Viterbi, 4 the chain's head on a lowest-priority stream
    of its own) taking mixed and uniform batches in turn on their own streams, as bench.py's
    pipelined mode does: every output equals a lone engine's."""
    m = txgen.make_mixed_fast(1024, min_len=64, max_len=2300, sigma=3.0, seed=81, device="cuda")
    u = txgen.make_batch(768, seed=82, sigma=4.0, device="cuda")
    S = max(m["max_nsym"], u["max_nsym"])
    ref = RxEngine(0)
    ref.reserve(1024, S)
    exp = {}
    for k, b in (("m", m), ("u", u)):
        pay, info = ref.rx(b["sym"], b["sym_off"], b["nsym"], S)
        exp[k] = (pay.cpu().numpy(), info.cpu().numpy())
    engs = [RxEngine(0), RxEngine(0)]
    for e in engs:
        e.reserve(1024, S)
    engs[0].link(engs[1], mode)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
    outs = []
    for i, k in enumerate("mumummuu"):
        b = m if k == "m" else u
        with torch.cuda.stream(streams[i % 2]):
            pay, info = engs[i % 2].rx(b["sym"], b["sym_off"], b["nsym"], S)
        outs.append((k, pay, info))
    torch.cuda.synchronize()
    for k, pay, info in outs:
        assert (pay.cpu().numpy() == exp[k][0]).all() and (info.cpu().numpy() == exp[k][1]).all(), k
    assert (exp["u"][1][:, 4] == 1).all()
    engs[0].link(engs[1], 0)


def test_chain_scrambler_states_and_short_payloads(engine, oracle):
    """The descrambler and CRC (k_descramble_crc) across scrambler states — every keystream
    phase the SERVICE field can announce, the stuck state 0 among them — and payload lengths
    around the kernel's boundaries (0..5 bytes: the plain-register path; 31..33, 255..257:
    chunk and dword edges; 2044: the largest): payloads and infos equal the oracle receiver's
    and, every CRC passing, the transmitted payloads."""
    states = np.arange(128) % 128
    for L, (mod, cod) in ((0, (0, 0)), (1, (1, 2)), (2, (3, 2)), (3, (2, 0)), (4, (3, 1)), (5, (0, 2)),
                          (31, (3, 2)), (32, (2, 2)), (33, (1, 0)), (255, (3, 2)), (256, (3, 1)), (257, (2, 0)),
                          (2044, (3, 2))):
        n = 128
        b = txgen.make_batch(n, mod=mod, coding=cod, payload_len=L, sigma=2.0, seed=300 + L, device="cuda",
                             scrambler=np.roll(states, L))
        engine.reserve(n, b["max_nsym"])
        pay, info = engine.rx(b["sym"], b["sym_off"], b["nsym"], b["max_nsym"])
        pay, info = pay.cpu().numpy(), info.cpu().numpy()
        sym = b["sym"].cpu().numpy()
        opay, res = oracle.rx_batch_time(sym, b["sym_off"].cpu().numpy(), b["nsym"].cpu().numpy())
        for i, r in enumerate(res):
            assert info[i, 2] == r["len"] == L + 4 and info[i, 4] == r["crc_ok"] == 1, (L, i)
            assert (pay[i, :L] == opay[i, :L]).all() and (pay[i, :L] == b["payload"][i]).all(), (L, i)


@pytest.mark.parametrize("mixed", [False, True])
def test_chain_plan_many_blocks(engine, mixed):
    """k_pkt_scan over more than 64 blocks of 1024 packets (its look-back crosses several
    64-record windows) and a partial last block: 66 x 1024 + 5 short packets, uniform (6 Mbps,
    20-byte payloads) or mixed (8 MCS, PSDU 8..120 B); every packet's CRC passes with the
    transmitted payload, so every offset, data-symbol prefix and wave start was right."""
    n = 66 * 1024 + 5
    if mixed:
        m = txgen.make_mixed_fast(n, min_len=8, max_len=120, sigma=2.0, seed=0x66, device="cuda", chunk=8192)
        lens = m["meta"][:, 2] - 4
        pays = m["payload"]
    else:
        m = txgen.make_batch(n, mod=0, coding=0, payload_len=20, sigma=2.0, seed=0x66, device="cuda", chunk=8192)
        lens = np.full(n, 20)
        pays = m["payload"]
    engine.reserve(n, m["max_nsym"])
    pay, info = engine.rx(m["sym"], m["sym_off"], m["nsym"], m["max_nsym"])
    pay, info = pay.cpu().numpy(), info.cpu().numpy()
    assert (info[:, 4] == 1).all(), np.nonzero(info[:, 4] != 1)[0][:10]
    for i in range(n):
        assert (pay[i, :lens[i]] == np.asarray(pays[i])[:lens[i]]).all(), i
    engine.plan_check()
