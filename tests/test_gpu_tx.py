"""GPU parity of the TX chain (transmitter.blk at 40 MHz) through the
C-ABI: bit-exact with the oracle on all 8 MCS and many lengths, the reference KAT, and a
loopback through the GPU receiver front end."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import ziria_amd as Z  # noqa: E402

MCS = [(0, 0), (0, 2), (1, 0), (1, 2), (2, 0), (2, 2), (3, 1), (3, 2)]


def _packets(oracle, n, seed):
    rng = np.random.default_rng(seed)
    pk = []
    for i in range(n):
        mod, cod = MCS[i % 8]
        ln = int(rng.choice([4, 5, 17, 100, 1000, 1504, 2048, int(rng.integers(4, 2049))]))
        pk.append(np.concatenate([oracle.plcp_header(mod, cod, ln), rng.integers(0, 256, ln - 4).astype(np.uint8)]))
    return pk


def test_tx_vs_oracle(oracle):
    pk = _packets(oracle, 64, 3)
    out, off = Z.wifi_tx_batch(pk)
    for i, p in enumerate(pk):
        exp = oracle.tx_packet(p)
        assert off[i + 1] - off[i] == exp.shape[0], i
        assert (out[off[i]:off[i + 1]] == exp).all(), i


def test_tx_kat_and_loopback(oracle, golden):
    fe = golden["ref_fe"]
    out, off = Z.wifi_tx_batch([fe["tx_in"]])
    o = out[off[0]:off[1]] * np.int16(10)                     # amp(10)
    assert (o[320:] == fe["tx_out"][320:]).all()                # see test_tx_oracle.test_tx_kat
    assert (o == oracle.tx_packet(fe["tx_in"]) * np.int16(10)).all()
    x = np.concatenate([np.zeros((1000, 2), np.int16), o])
    pay, info, det, nok = Z.wifi_rx_stream_batch(x, np.array([0, x.shape[0]], np.int32), downsample=True)
    assert nok == 1 and (pay[0, :96] == fe["tx_in"][3:]).all()
