"""TX chain: the oracle's transmitter() against the reference KAT
code/WiFi/tests/test_tx and IFFT<128> vectors of the compiled reference brick."""
import ctypes as C

import numpy as np
import pytest


@pytest.fixture(scope="module")
def fe(golden):
    return golden["ref_fe"]


def test_ifft128_reference_vectors(oracle, fe):
    for a, b in zip(fe["ifft128_in"], fe["ifft128_out"]):
        assert (oracle.ifft128(a) == b).all()


def test_tx_kat(oracle, fe):
    """test_tx: read >>> bits >>> transmitter >>> amp(10).  Exact on the LTS, SIGNAL and data
    symbols; the STS differs by one LSB on 40 of its 320 samples: the ground was made with
    sts_mod = 15780, while createPreamble.blk:25 computes int16(10720 * 1.472) = 15779 (wplc
    truncates double -> int16, src/Codegen/CgValDom.hs:86 and the constant folder,
    src/Optimize/Interpreter.hs:1851)."""
    o = oracle.tx_packet(fe["tx_in"]).astype(np.int16) * np.int16(10)
    g = fe["tx_out"]
    assert o.shape == g.shape
    assert (o[320:] == g[320:]).all()
    d = np.abs(o[:320].astype(np.int64) - g[:320])
    assert d.max() <= 10 and int((d.max(1) > 0).sum()) == 40


def test_plcp_header_bytes(oracle, fe):
    assert (oracle.plcp_header(1, 2, 100) == fe["tx_in"][:3]).all()


def test_tx_loopback_oracle(oracle, fe):
    """TX (test_tx input) x10 >>> append_idle >>> downSample >>> receiver() gives the payload."""
    o = oracle.tx_packet(fe["tx_in"]).astype(np.int16) * np.int16(10)
    x = oracle.downsample(np.concatenate([np.zeros((1000, 2), np.int16), o]))
    pay, r, det, co, d0 = oracle.rx_stream(x)
    assert r["crc_ok"] == 1 and (pay == fe["tx_in"][3:]).all()


def test_engine_host_tx_preamble(oracle):
    import ziria_amd as Z
    from ziria_amd import build
    build.build()
    a = np.zeros((640, 2), np.int16)
    assert Z.lib().zrx_tx_preamble(a.ctypes.data_as(C.c_void_p)) == 0
    assert (a == oracle.tx_preamble()).all()
    h = oracle.plcp_header(3, 2, 1504)
    assert Z.lib().zrx_tx_samples(h.ctypes.data_as(C.c_void_p)) == 640 + 160 * 57
