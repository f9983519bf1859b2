"""GPU parity of the RX front end (downSample, removeDC, cca, LTS,
DataSymbol, then the decode chain with ChannelEqualization + PilotTrack) through the C-ABI:
the reference's end-to-end KATs and capture variants against the oracle.  Bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import ziria_amd as Z  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402
from tests import fe_cases  # noqa: E402

DET = ("noSamples", "shift", "energy", "noise", "maxCorr")


@pytest.fixture(scope="module")
def fe(golden):
    return golden["ref_fe"]


def test_receiver_kats_host_api(fe):
    """test_rx (append_idle >>> downSample >>> receiver) and test_real_rx (an over-the-air
    capture, append_idle x10 >>> receiver) in one batch of two captures."""
    rx, real = fe_cases.kat_streams(fe)
    for x, ds, exp in ((rx, True, fe["rx_out"]), (real, False, fe["real_out"])):
        pay, info, det, nok = Z.wifi_rx_stream_batch(x, np.array([0, x.shape[0]], np.int32), downsample=ds)
        assert det[0, 0] == 1 and info["crc_ok"][0] == 1 and nok == 1
        assert (pay[0, :exp.size] == exp).all()


def test_capture_variants_vs_oracle(oracle, fe):
    caps = fe_cases.variants(fe, 120, seed=23)
    off = np.cumsum([0] + [c.shape[0] for c in caps]).astype(np.int64)
    x = torch.from_numpy(np.concatenate(caps)).cuda()
    e = RxEngine(0)
    pay, info, det = e.rx_stream(x, torch.from_numpy(off[:-1]).cuda(),
                                 torch.from_numpy(np.diff(off).astype(np.int32)).cuda(), int(np.diff(off).max()))
    pay, info, det = pay.cpu().numpy(), info.cpu().numpy(), det.cpu().numpy()
    e.close()
    decoded = 0
    for i, c in enumerate(caps):
        opay, r, odet, co, d0 = oracle.rx_stream(c)
        if r["ret"] == -1:                                # nothing detected
            assert det[i, 0] == 0, i
            continue
        assert det[i, 0] == 1, i
        assert tuple(det[i, 1:6]) == tuple(odet[k] for k in DET), (i, det[i], odet)
        if r["ret"] != 0:
            continue
        assert (info[i, 0], info[i, 1], info[i, 2], info[i, 3]) == (r["modulation"], r["coding"], r["len"], r["err"]), i
        assert info[i, 4] == r["crc_ok"], i
        L = max(r["len"] - 4, 0)
        assert (pay[i, :L] == opay[:L]).all(), i
        decoded += r["crc_ok"]
    assert decoded >= 60
