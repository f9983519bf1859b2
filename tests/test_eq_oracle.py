"""ChannelEqualization + PilotTrack: the oracle restatement against
the reference's KATs (receiver/tests/test_c_{PilotTrack,ChannelEqualization}), the
reference integer trigonometry (hashes / samples in tests/golden/ref_eq.npz) and the
reference-brick fixtures; the engine's host-side trig tables against the same hashes."""
import ctypes as C
import hashlib

import numpy as np
import pytest


@pytest.fixture(scope="module")
def eq(golden):
    return golden["ref_eq"]


def test_pilot_track_kat(oracle, eq):
    x, g = eq["pilot_kat_in"], eq["pilot_kat_out"]
    for k in range(x.shape[0]):                  # one PilotTrack instance over the stream
        assert (oracle.pilot_track(x[k], k) == g[k]).all(), k


def test_channel_eq_kat(oracle, eq):
    co = np.tile(np.array([2, 2], np.int16), (64, 1))      # test_c_ChannelEqualization.blk:26-28
    x, g = eq["cheq_kat_in"], eq["cheq_kat_out"]
    for k in range(x.shape[0]):
        assert (oracle.channel_eq(x[k], co) == g[k]).all(), k


def test_trig_tables_match_reference(oracle, eq):
    s, c, a = oracle.trig_tables()
    assert hashlib.sha256(s.tobytes()).hexdigest() == str(eq["sin_sha256"])
    assert hashlib.sha256(c.tobytes()).hexdigest() == str(eq["cos_sha256"])


def test_atan2_reference_samples(oracle, eq):
    yx, out = eq["atan2_yx"], eq["atan2_out"]
    got = np.array([oracle.atan2_16(y, x) for y, x in yx], np.int16)
    assert (got == out).all()


def test_atan2_reference_grid(oracle, eq):
    lo, hi = (int(v) for v in eq["atan2_grid_lo_hi"])
    g = np.arange(lo, hi + 1)
    got = np.array([[oracle.atan2_16(y, x) for x in g] for y in g], np.int16)
    assert hashlib.sha256(got.tobytes()).hexdigest() == str(eq["atan2_grid_sha256"])


def test_pilot_sign_is_reference_table(oracle):
    # the 802.11a polarity sequence with the reference tables' +1 at entry 52
    s = [oracle.lib().zo_pilot_sign(m) for m in range(128)]
    assert s[:8] == [0, 0, 0, -1, -1, -1, 0, -1] and s[52] == 0 and s[126:] == [0, 0]


def test_ofdm_eq_symbols_fixture(oracle, eq):
    x, ch, out, k = eq["eqsym_in"], eq["eqsym_chan"], eq["eqsym_out"], eq["eqsym_k"]
    for i in range(x.shape[0]):
        assert (oracle.ofdm_eq_symbol(x[i], ch[i // 150], k[i]) == out[i]).all(), i


def test_eq_chain_fixture(oracle, eq):
    pay, res = oracle.rx_batch_time_eq(eq["eq_sym"], eq["eq_off"], eq["eq_nsym"], eq["eq_chan"], nthreads=4)
    po = eq["eq_payload_off"]
    for i, r in enumerate(res):
        assert (r["modulation"], r["coding"], r["len"]) == tuple(eq["eq_meta"][i])
        assert r["crc_ok"] == eq["eq_crc"][i], i
        e = eq["eq_payload"][po[i]:po[i + 1]]
        assert (pay[i, :e.size] == e).all(), i


def test_engine_host_trig_tables(oracle, eq):
    """The engine builds its device tables from the same closed forms (host code, no GPU);
    the oracle's tables are pinned to the reference by the tests above."""
    import ziria_amd as Z
    from ziria_amd import build
    build.build()
    s, c, a = (np.zeros(65536, np.int16) for _ in range(3))
    p = lambda v: v.ctypes.data_as(C.c_void_p)   # noqa: E731
    assert Z.lib().zrx_trig_tables(p(s), p(c), p(a)) == 0
    assert hashlib.sha256(s.tobytes()).hexdigest() == str(eq["sin_sha256"])
    assert hashlib.sha256(c.tobytes()).hexdigest() == str(eq["cos_sha256"])
    assert (a == oracle.trig_tables()[2]).all()
