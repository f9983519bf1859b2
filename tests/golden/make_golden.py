"""Generates the committed golden fixtures in tests/golden/ (run in the dev container,
where /root/reference exists; the GPU box only reads the .npz files).

Sources, in order of authority:
  1. the reference's own known-answer tests, copied as DATA (inputs + expected outputs):
     tests/libs/test_fft.{infile,outfile.ground} (FFT64 block),
     code/WiFi/receiver/tests/testViterbi{,Sig11a}.{infile,outfile.ground},
     code/WiFi/tests/test_encdec_{6,12,18,24,36}mbps.{infile,outfile.ground};
  2. tables parsed from the reference .blk sources (demap LUTs const.blk:74-150,
     deinterleaver tables Deinterleave*.blk) = expected outputs of those blocks on
     identity/index inputs;
  3. outputs of the reference bricks compiled here from /root/reference/csrc
     (oracle/_ref/libzref.so via oracle/Makefile.ref): FFT64, Viterbi (all rates), SIGNAL.
     The .blk glue around them (demap, deinterleave, descramble, CRC) has no C form in the
     reference (wplc is unavailable), so chain fixtures use the reference FFT + Viterbi
     bricks with the oracle's glue, which is itself pinned by the encdec KATs above.

  4. ref_fftn.npz: the whole tests/libs/test_fft KAT (all 42 sizes of __ext_sora_fft) and
     the compiled reference FFT brick on random, saturating and small vectors of every size.

Usage: python tests/golden/make_golden.py        (all fixtures)
       python tests/golden/make_golden.py fftn   (ref_fftn.npz only)
       python tests/golden/make_golden.py eq     (ref_eq.npz only)
       python tests/golden/make_golden.py fe     (ref_fe.npz only)
"""
import ctypes as C
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from tests.golden import synth  # noqa: E402

REF = "/root/reference"
W = REF + "/code/WiFi"


def rd(p):
    txt = open(p).read().replace("\n", ",")
    return np.array([int(v) for v in txt.split(",") if v.strip() != ""], np.int64)


def ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def ref_fft64(R, x):
    out = np.zeros_like(x)
    for i in range(x.shape[0]):
        xi = np.ascontiguousarray(x[i])
        oi = np.zeros_like(xi)
        R.zref_sora_fft(ptr(oi), 64, ptr(xi))
        out[i] = oi
    return out


def ref_viterbi(R, soft, frame_len, code_rate, chunk=48):
    R.zref_viterbi_init(frame_len, code_rate, 256)
    buf = np.zeros(12000, np.uint8)
    outs = []
    for i in range(0, soft.size, chunk):
        s = np.ascontiguousarray(soft[i:i + chunk], np.int8)
        bits = R.zref_viterbi_decode(ptr(s), s.size, ptr(buf), 96000)
        outs.append(buf[: bits // 8].copy())
    return np.concatenate(outs) if outs else np.zeros(0, np.uint8)


def ref_sig(R, soft48):
    s = np.ascontiguousarray(soft48, np.int8)
    o = np.zeros(4, np.uint8)
    R.zref_viterbi_sig(ptr(s), ptr(o))
    b = np.unpackbits(o, bitorder="little")[:24].copy()
    b[18:] = 0
    return np.packbits(b, bitorder="little")


def kats():
    d = {}
    inp = rd(REF + "/tests/libs/test_fft.infile")
    gnd = rd(REF + "/tests/libs/test_fft.outfile.ground")
    off = sum([12, 16, 24, 32, 36, 48, 60])          # FFT64 is the 8th block of test_fft.wpl
    d["fft64_kat_in"] = inp[2 * off:2 * off + 128].reshape(64, 2).astype(np.int16)
    d["fft64_kat_out"] = gnd[2 * off:2 * off + 128].reshape(64, 2).astype(np.int16)
    d["vit_kat_soft"] = rd(W + "/receiver/tests/testViterbi.infile").astype(np.int8)
    d["vit_kat_bits"] = rd(W + "/receiver/tests/testViterbi.outfile.ground").astype(np.uint8)
    d["sig_kat_soft"] = rd(W + "/receiver/tests/testViterbiSig11a.infile")[:48].astype(np.int8)
    d["sig_kat_bits"] = rd(W + "/receiver/tests/testViterbiSig11a.outfile.ground").astype(np.uint8)
    for r in (6, 12, 18, 24, 36):
        base = W + f"/tests/test_encdec_{r}mbps"
        d[f"encdec_{r}_in"] = rd(base + ".infile").astype(np.int8)
        d[f"encdec_{r}_out"] = rd(base + ".outfile.ground").astype(np.int8)
    return d


def tables():
    src = open(W + "/const.blk").read()
    d = {}
    for name in ("m_bpsk_lut", "m_qam16_lut2", "m_qam64_lut2", "m_qam64_lut3"):
        m = re.search(r"let\s+" + name + r"\s*=\s*\{([^}]*)\}", src)
        d[name] = np.array([int(v) for v in m.group(1).replace("\n", " ").split(",")], np.uint8)
    for mod, tag in enumerate(("BPSK", "QPSK", "QAM16", "QAM64")):
        t = open(W + f"/receiver/decoding/Deinterleave{tag}.blk").read()
        pairs = re.findall(r"output\[(\d+)\]\s*:=\s*symbol\[(\d+)\]", t)
        n = len(pairs)
        perm = np.zeros(n, np.int32)
        for o, i in pairs:
            perm[int(o)] = int(i)
        d[f"deint_{mod}"] = perm
    return d


def fft_vectors(R, n=1024, seed=0xF64):
    rng = np.random.default_rng(seed)
    x = np.empty((n, 64, 2), np.int16)
    x[: n // 4] = rng.integers(-32768, 32768, (n // 4, 64, 2))
    x[n // 4: n // 2] = rng.choice(np.array([-32768, -32767, 32767, 0, 1, -1], np.int16),
                                  (n // 4, 64, 2))
    x[n // 2:] = rng.integers(-2500, 2500, (n - n // 2, 64, 2))
    return {"fft_in": x, "fft_out": ref_fft64(R, x)}


def viterbi_vectors(R):
    d = {}
    cases = []
    for cr in (0, 1, 2):
        for fl in (1, 3, 100, 333, 1500, 4095):
            for noise in (0, 3, 7, -1):          # -1: uniformly random soft values
                cases.append((cr, fl, noise))
    softs, offs, outs, ooffs = [], [0], [], [0]
    for idx, (cr, fl, noise) in enumerate(cases):
        s = synth.viterbi_soft(cr, fl, noise, seed=0x5EED + idx)
        o = ref_viterbi(R, s, fl, cr)
        softs.append(s)
        offs.append(offs[-1] + s.size)
        outs.append(o)
        ooffs.append(ooffs[-1] + o.size)
    d["vit_cases"] = np.array(cases, np.int32)
    d["vit_soft"] = np.concatenate(softs).astype(np.int8)
    d["vit_soft_off"] = np.array(offs, np.int64)
    d["vit_out"] = np.concatenate(outs).astype(np.uint8)
    d["vit_out_off"] = np.array(ooffs, np.int64)
    # adversarial: patterns that drive metrics toward u8 wrap
    adv = np.tile(np.array([0, 7, 7, 0, 0, 0, 7, 7, 7, 7, 0, 0], np.int8), 800)[: 48 * 200]
    for cr in (0, 1, 2):
        d[f"vit_adv_out_{cr}"] = ref_viterbi(R, adv, 1000, cr)
    d["vit_adv_soft"] = adv
    rng = np.random.default_rng(0x516)
    sig = rng.integers(0, 8, (256, 48)).astype(np.int8)
    d["sig_soft"] = sig
    d["sig_bits"] = np.stack([ref_sig(R, s) for s in sig])
    return d


def chain_vectors(R):
    """54 Mbps time-domain packets (config 3 shape, few packets) and a mixed-MCS batch."""
    d = {}
    for tag, plan in (("c54", synth.plan_54mbps(8, 1500)), ("mix", synth.plan_mixed(16, max_len=700))):
        sym, off, nsym, meta = synth.packets_time(plan, seed=0xC0DE if tag == "c54" else 0x4D1)
        pays, crcs = [], []
        for p in range(len(off)):
            x = sym[off[p]: off[p] + nsym[p]]
            f = ref_fft64(R, x)                                   # reference FFT brick
            sub = np.stack([O.get_data(fi) for fi in f])
            # reference Viterbi brick for the data decode, oracle glue around it
            pay, ok = ref_chain_from_freq(R, sub)
            pays.append(pay)
            crcs.append(ok)
        d[f"{tag}_sym"] = sym
        d[f"{tag}_off"] = off
        d[f"{tag}_nsym"] = nsym
        d[f"{tag}_meta"] = meta
        d[f"{tag}_payload"] = np.concatenate(pays)
        d[f"{tag}_payload_off"] = np.cumsum([0] + [p.size for p in pays]).astype(np.int64)
        d[f"{tag}_crc"] = np.array(crcs, np.int32)
    return d


def ref_chain_from_freq(R, sub):
    lim = O.demap_limit(sub[0])
    soft = O.deinterleave(0, O.demap(0, lim))
    hb = ref_sig(R, soft)
    h = O.parse_header(hb)
    mod, cod, ln = h["modulation"], h["coding"], h["len"]
    R.zref_viterbi_init(ln + 2, cod, 256)
    buf = np.zeros(12000, np.uint8)
    dec = []
    total = 0
    for k in range(1, sub.shape[0]):
        if total >= (ln + 2) * 8:
            break
        s = O.deinterleave(mod, O.demap(mod, O.demap_limit(sub[k])))
        for c in range(0, s.size, 48):
            ss = np.ascontiguousarray(s[c:c + 48])
            bits = R.zref_viterbi_decode(ptr(ss), 48, ptr(buf), 96000)
            dec.append(buf[: bits // 8].copy())
            total += bits
    dec = np.concatenate(dec)
    pay, ok = O.descramble_crc(dec, ln)
    return pay, int(ok)


def eq_vectors(R):
    """ChannelEqualization + PilotTrack: the reference KATs
    receiver/tests/test_c_{PilotTrack,ChannelEqualization}.{infile,outfile.ground} as data,
    hashes and samples of the reference integer trigonometry (csrc/intalgx.h via the
    compiled reference), per-symbol FFT >>> ChannelEqualization >>> PilotTrack outputs
    (reference FFT brick, restated .blk glue pinned by those KATs), and a packet batch
    through a frequency-selective channel decoded with the reference FFT + Viterbi bricks."""
    import hashlib
    d = {}
    T = W + "/receiver/tests/"
    for tag, name in (("pilot", "test_c_PilotTrack"), ("cheq", "test_c_ChannelEqualization")):
        g = rd(T + name + ".outfile.ground")
        n = g.size // 128
        d[f"{tag}_kat_in"] = rd(T + name + ".infile")[: n * 128].reshape(n, 64, 2).astype(np.int16)
        d[f"{tag}_kat_out"] = g.reshape(n, 64, 2).astype(np.int16)
    sv = np.array([R.zref_sin16(int(np.int16(np.uint16(r)))) for r in range(65536)], np.int16)
    cv = np.array([R.zref_cos16(int(np.int16(np.uint16(r)))) for r in range(65536)], np.int16)
    d["sin_sha256"] = np.array(hashlib.sha256(sv.tobytes()).hexdigest())
    d["cos_sha256"] = np.array(hashlib.sha256(cv.tobytes()).hexdigest())
    grid = np.arange(-300, 301)
    ag = np.array([[R.zref_atan2_16(int(y), int(x)) for x in grid] for y in grid], np.int16)
    d["atan2_grid_lo_hi"] = np.array([-300, 300], np.int32)
    d["atan2_grid_sha256"] = np.array(hashlib.sha256(ag.tobytes()).hexdigest())
    rng = np.random.default_rng(0xA7A2)
    edge = np.array([0, 1, -1, 63, 64, -64, -65, 127, 128, -128, -129, 255, -255, 256, -256,
                     32767, -32768, -32767, 16384, -16384], np.int64)
    yx = np.concatenate([rng.integers(-32768, 32768, (20000, 2)),
                         np.stack(np.meshgrid(edge, edge), -1).reshape(-1, 2)])
    d["atan2_yx"] = yx.astype(np.int16)
    d["atan2_out"] = np.array([R.zref_atan2_16(int(y), int(x)) for y, x in yx], np.int16)
    # symbol level: random, extreme and realistic symbols, per-packet coefficients
    x = np.empty((600, 64, 2), np.int16)
    x[:200] = rng.integers(-32768, 32768, (200, 64, 2))
    x[200:300] = rng.choice(np.array([-32768, -32767, 32767, 0, 1, -1], np.int16), (100, 64, 2))
    x[300:] = rng.integers(-2500, 2500, (300, 64, 2))
    chan = rng.integers(-32768, 32768, (4, 64, 2)).astype(np.int16)   # 4 packets x 150 symbols
    chan[1] = rng.integers(-600, 600, (64, 2))
    chan[2] = rng.choice(np.array([-32768, 32767, 0, 256, -256], np.int16), (64, 2))
    f = ref_fft64(R, x)
    out = np.zeros_like(x)
    L = O.lib()
    for i in range(600):
        e = np.zeros((64, 2), np.int16)
        L.zo_channel_eq(ptr(np.ascontiguousarray(f[i])), ptr(np.ascontiguousarray(chan[i // 150])), ptr(e))
        o = np.zeros((64, 2), np.int16)
        L.zo_pilot_track(ptr(e), i % 150, ptr(o))      # symbol index within its packet (wraps at 128)
        out[i] = o
    d["eqsym_in"], d["eqsym_chan"], d["eqsym_out"] = x, chan, out
    d["eqsym_k"] = np.array([i % 150 for i in range(600)], np.int32)
    # packets through a channel
    plan = synth.plan_mixed(20, max_len=1200, seed=0xE9) + synth.plan_54mbps(4, 1500)
    sym, off, nsym, meta, chan = synth.packets_time_eq(plan, seed=0xE90)
    pays, crcs = [], []
    for p in range(len(off)):
        f = ref_fft64(R, sym[off[p]: off[p] + nsym[p]])
        sub = []
        for k in range(f.shape[0]):
            e = np.zeros((64, 2), np.int16)
            L.zo_channel_eq(ptr(np.ascontiguousarray(f[k])), ptr(np.ascontiguousarray(chan[p])), ptr(e))
            o = np.zeros((64, 2), np.int16)
            L.zo_pilot_track(ptr(e), k, ptr(o))
            sub.append(O.get_data(o))
        pay, ok = ref_chain_from_freq(R, np.stack(sub))
        pays.append(pay)
        crcs.append(ok)
    d["eq_sym"], d["eq_off"], d["eq_nsym"], d["eq_meta"], d["eq_chan"] = sym, off, nsym, meta, chan
    d["eq_payload"] = np.concatenate(pays)
    d["eq_payload_off"] = np.cumsum([0] + [p.size for p in pays]).astype(np.int64)
    d["eq_crc"] = np.array(crcs, np.int32)
    return d


def fe_vectors(R):
    """RX front end: the reference's end-to-end KATs
    code/WiFi/tests/test_rx.* and test_real_rx.* (captures -> decoded bytes) and the block
    KATs receiver/tests/test_c_{RemoveDC,DownSample,DataSymbol,LTS} as data, plus IFFT64
    vectors of the compiled reference brick (the STS pattern of cca_tufv.blk)."""
    d = {}
    for tag, name in (("rx", "test_rx"), ("real", "test_real_rx")):
        d[f"{tag}_in"] = rd(W + f"/tests/{name}.infile").reshape(-1, 2).astype(np.int16)
        d[f"{tag}_out"] = rd(W + f"/tests/{name}.outfile.ground").astype(np.int8).view(np.uint8)
    d["tx_in"] = rd(W + "/tests/test_tx.infile").astype(np.int8).view(np.uint8)
    d["tx_out"] = rd(W + "/tests/test_tx.outfile.ground").reshape(-1, 2).astype(np.int16)
    x = np.zeros((40, 128, 2), np.int16)                 # IFFT<128> vectors (the TX's 40 MHz IFFT)
    rng0 = np.random.default_rng(0x128)
    x[:20] = rng0.integers(-32768, 32768, (20, 128, 2))
    x[20:] = rng0.choice(np.array([-32768, 32767, 0, 10720, -10720], np.int16), (20, 128, 2))
    o = np.zeros_like(x)
    for i in range(40):
        xi = np.ascontiguousarray(x[i])
        oi = np.zeros_like(xi)
        R.zref_sora_ifft128(ptr(oi), ptr(xi))
        o[i] = oi
    d["ifft128_in"], d["ifft128_out"] = x, o
    T = W + "/receiver/tests/"
    for tag, name in (("rdc", "test_c_RemoveDC"), ("ds", "test_c_DownSample"), ("dsym", "test_c_DataSymbol"),
                      ("lts", "test_c_LTS")):
        x = rd(T + name + ".infile")
        d[f"{tag}_in"] = x[: x.size // 2 * 2].reshape(-1, 2).astype(np.int16)
        d[f"{tag}_out"] = rd(T + name + ".outfile.ground").reshape(-1, 2).astype(np.int16)
    rng = np.random.default_rng(0x1FF7)
    x = np.empty((200, 64, 2), np.int16)
    x[:100] = rng.integers(-32768, 32768, (100, 64, 2))
    x[100:150] = rng.choice(np.array([-32768, 32767, 0, 1, -1], np.int16), (50, 64, 2))
    x[150:] = rng.integers(-3000, 3000, (50, 64, 2))
    out = np.zeros_like(x)
    for i in range(200):
        xi = np.ascontiguousarray(x[i])
        oi = np.zeros_like(xi)
        R.zref_sora_ifft64(ptr(oi), ptr(xi))
        out[i] = oi
    d["ifft_in"], d["ifft_out"] = x, out
    return d


def fftn_vectors(R, per=6, seed=0xFF7):
    """test_fft KAT (test_fft.wpl: one block per size, in O.FFT_SIZES order) + reference
    brick outputs for `per` vectors of every size, concatenated (offsets in vec_off)."""
    d = {}
    inp = rd(REF + "/tests/libs/test_fft.infile")
    gnd = rd(REF + "/tests/libs/test_fft.outfile.ground")
    tot = sum(O.FFT_SIZES)
    d["sizes"] = np.array(O.FFT_SIZES, np.int32)
    d["kat_in"] = inp[: 2 * tot].reshape(tot, 2).astype(np.int16)
    d["kat_out"] = gnd[: 2 * tot].reshape(tot, 2).astype(np.int16)
    rng = np.random.default_rng(seed)
    xs, ys, off = [], [], [0]
    for n in O.FFT_SIZES:
        for t in range(per):
            if t < 2:
                x = rng.integers(-32768, 32768, (n, 2))
            elif t < 4:
                x = rng.choice(np.array([-32768, -32767, 32767, 0, 1, -1]), (n, 2))
            else:
                x = rng.integers(-3000, 3000, (n, 2))
            x = np.ascontiguousarray(x, np.int16)
            y = np.zeros_like(x)
            R.zref_sora_fft(ptr(y), n, ptr(x))
            xs.append(x); ys.append(y); off.append(off[-1] + n)
    d["vec_in"], d["vec_out"] = np.concatenate(xs), np.concatenate(ys)
    d["vec_off"], d["vec_per"] = np.array(off, np.int64), np.int32(per)
    return d


def main():
    O.build()
    R = O.ref()
    assert R is not None, "reference bricks not built (needs /root/reference)"
    if sys.argv[1:] == ["fe"]:
        np.savez_compressed(os.path.join(HERE, "ref_fe.npz"), **fe_vectors(R))
        print("ref_fe.npz", os.path.getsize(os.path.join(HERE, "ref_fe.npz")))
        return
    if sys.argv[1:] == ["fftn"]:
        np.savez_compressed(os.path.join(HERE, "ref_fftn.npz"), **fftn_vectors(R))
        print("ref_fftn.npz", os.path.getsize(os.path.join(HERE, "ref_fftn.npz")))
        return
    if sys.argv[1:] == ["eq"]:
        np.savez_compressed(os.path.join(HERE, "ref_eq.npz"), **eq_vectors(R))
        print("ref_eq.npz", os.path.getsize(os.path.join(HERE, "ref_eq.npz")))
        return
    np.savez_compressed(os.path.join(HERE, "ref_kats.npz"), **kats())
    np.savez_compressed(os.path.join(HERE, "ref_tables.npz"), **tables())
    np.savez_compressed(os.path.join(HERE, "ref_fft64.npz"), **fft_vectors(R))
    np.savez_compressed(os.path.join(HERE, "ref_viterbi.npz"), **viterbi_vectors(R))
    np.savez_compressed(os.path.join(HERE, "ref_chain.npz"), **chain_vectors(R))
    np.savez_compressed(os.path.join(HERE, "ref_eq.npz"), **eq_vectors(R))
    np.savez_compressed(os.path.join(HERE, "ref_fe.npz"), **fe_vectors(R))
    np.savez_compressed(os.path.join(HERE, "ref_fftn.npz"), **fftn_vectors(R))
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
