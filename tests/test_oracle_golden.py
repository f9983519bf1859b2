"""The oracle (scalar C restatement) against the reference's own known-answer tests and
the golden fixtures produced by the compiled reference bricks (tests/golden/)."""
import zlib

import numpy as np
import pytest


def test_fft64_kat(oracle, golden):
    k = golden["ref_kats"]
    assert (oracle.fft64(k["fft64_kat_in"]) == k["fft64_kat_out"]).all()


def test_fft64_reference_vectors(oracle, golden):
    g = golden["ref_fft64"]
    assert (oracle.fft64(g["fft_in"]) == g["fft_out"]).all()


def test_fft_all_sizes_kat(oracle, golden):
    """tests/libs/test_fft (one block of every __ext_sora_fft size, 12..2048)."""
    g = golden["ref_fftn"]
    off = 0
    for n in g["sizes"]:
        n = int(n)
        assert (oracle.fft_n(n, g["kat_in"][off:off + n]) == g["kat_out"][off:off + n]).all(), n
        off += n


def test_fft_all_sizes_reference_vectors(oracle, golden):
    """Reference FFT brick outputs on random, saturating and small vectors of every size."""
    g = golden["ref_fftn"]
    o, per = g["vec_off"], int(g["vec_per"])
    for i, n in enumerate(g["sizes"]):
        for t in range(per):
            a, b = o[i * per + t], o[i * per + t + 1]
            assert (oracle.fft_n(int(n), g["vec_in"][a:b]) == g["vec_out"][a:b]).all(), (int(n), t)


def test_fft_unsupported_sizes(oracle):
    for n in (0, 8, 20, 63, 100, 4096):
        with pytest.raises(ValueError):
            oracle.fft_n(n, np.zeros((max(n, 1), 2), np.int16))


def test_demap_tables(oracle, golden):
    t = golden["ref_tables"]
    L = oracle.luts()
    for i, n in enumerate(("m_bpsk_lut", "m_qam16_lut2", "m_qam64_lut2", "m_qam64_lut3")):
        assert (L[i] == t[n]).all(), n


@pytest.mark.parametrize("mod", [0, 1, 2, 3])
def test_deinterleave_tables(oracle, golden, mod):
    assert (oracle.deint_perm(mod) == golden["ref_tables"][f"deint_{mod}"]).all()


def test_viterbi_kat(oracle, golden):
    k = golden["ref_kats"]
    out = oracle.viterbi_decode(k["vit_kat_soft"], 100, 0)
    assert (np.unpackbits(out, bitorder="little") == k["vit_kat_bits"]).all()


def test_signal_kat(oracle, golden):
    k = golden["ref_kats"]
    w = oracle.viterbi_sig(k["sig_kat_soft"])
    b = np.unpackbits(w, bitorder="little")[:24].copy()
    b[18:] = 0
    assert (b == k["sig_kat_bits"]).all()


def test_viterbi_reference_frames(oracle, golden):
    g = golden["ref_viterbi"]
    so, oo = g["vit_soft_off"], g["vit_out_off"]
    for i, (cr, fl, noise) in enumerate(g["vit_cases"]):
        out = oracle.viterbi_decode(g["vit_soft"][so[i]:so[i + 1]], int(fl), int(cr))
        assert (out == g["vit_out"][oo[i]:oo[i + 1]]).all(), (cr, fl, noise)


def test_viterbi_adversarial(oracle, golden):
    g = golden["ref_viterbi"]
    for cr in (0, 1, 2):
        assert (oracle.viterbi_decode(g["vit_adv_soft"], 1000, cr) == g[f"vit_adv_out_{cr}"]).all()


def test_signal_reference_vectors(oracle, golden):
    g = golden["ref_viterbi"]
    for s, exp in zip(g["sig_soft"], g["sig_bits"]):
        b = np.unpackbits(oracle.viterbi_sig(s), bitorder="little")[:24].copy()
        b[18:] = 0
        assert (np.packbits(b, bitorder="little") == exp).all()


def test_crc_is_zlib(oracle):
    rng = np.random.default_rng(0)
    for n in (0, 1, 3, 100, 1500, 4091):
        b = rng.integers(0, 256, n).astype(np.uint8)
        assert oracle.crc32_bits(b) == zlib.crc32(b.tobytes())


def _encdec_sub(oracle, d, perm):
    hb = (d[:3] & 0xFF).astype(np.uint8)
    h = oracle.parse_header(hb)
    coded = oracle.tx_encode(np.unpackbits(hb, bitorder="little")[:24], 0)
    il = np.zeros(48, np.uint8)
    il[perm] = coded
    sig = np.stack([np.where(il == 1, 10720, -10720), np.zeros(48)], 1).astype(np.int16)
    pay = (d[3:3 + h["len"] - 4] & 0xFF).astype(np.uint8)
    sub = oracle.tx_packet_freq(pay, h["modulation"], h["coding"])
    sub[0] = sig
    return np.trunc(sub.astype(np.int32) / 80).astype(np.int16)     # encdec_atten(16*5)


@pytest.mark.parametrize("rate", [6, 12, 18, 24, 36])
def test_encdec_kats(oracle, golden, rate):
    """code/WiFi/tests/test_encdec.blk: TX -> /80 -> receiveBits; ground = payload bytes."""
    k = golden["ref_kats"]
    sub = _encdec_sub(oracle, k[f"encdec_{rate}_in"].astype(np.int64), oracle.deint_perm(0))
    pay, r = oracle.rx_packet_freq(sub)
    assert r["crc_ok"] == 1
    assert (pay.astype(np.int8) == k[f"encdec_{rate}_out"]).all()


@pytest.mark.parametrize("tag", ["c54", "mix"])
def test_chain_reference_packets(oracle, golden, tag):
    g = golden["ref_chain"]
    pay, res = oracle.rx_batch_time(g[f"{tag}_sym"], g[f"{tag}_off"], g[f"{tag}_nsym"], nthreads=4)
    po = g[f"{tag}_payload_off"]
    for i in range(len(res)):
        assert res[i]["crc_ok"] == g[f"{tag}_crc"][i]
        e = g[f"{tag}_payload"][po[i]:po[i + 1]]
        assert (pay[i, :e.size] == e).all()
