"""GPU parity of ChannelEqualization + PilotTrack (receiver.blk:66-71)
through the C-ABI: against the reference-pinned fixtures (tests/golden/ref_eq.npz) and the
oracle on random and full-size batches.  Integer work: bit-exact, no tolerance."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import ziria_amd as Z  # noqa: E402
from ziria_amd import txgen  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402
from tests.golden import synth  # noqa: E402


@pytest.fixture(scope="module")
def engine():
    e = RxEngine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def eq(golden):
    return golden["ref_eq"]


def test_ofdm_eq_fixture(engine, eq):
    """FFT >>> ChannelEqualization >>> PilotTrack, 4 packets x 150 symbols (pilot index wraps),
    random / extreme / realistic symbols and coefficients."""
    x = torch.from_numpy(eq["eqsym_in"]).cuda()
    off = torch.arange(4, dtype=torch.int64).cuda() * 150
    ns = torch.full((4,), 150, dtype=torch.int32).cuda()
    ch = torch.from_numpy(eq["eqsym_chan"]).cuda().contiguous()
    out = engine.ofdm_eq(x, off, ns, ch).cpu().numpy()
    assert (out == eq["eqsym_out"]).all()


def test_ofdm_eq_pilot_kat(engine, eq):
    """Realistic symbols (the first 150 of the PilotTrack KAT input, fed as time-domain
    samples) with unit-gain coefficients (256 at norm_shift 8), against the oracle."""
    from oracle import oracle as O
    x = eq["pilot_kat_in"][:150]
    ch = np.zeros((1, 64, 2), np.int16)
    ch[..., 0] = 256
    out = engine.ofdm_eq(torch.from_numpy(x).cuda(), torch.zeros(1, dtype=torch.int64).cuda(),
                         torch.full((1,), 150, dtype=torch.int32).cuda(), torch.from_numpy(ch).cuda()).cpu().numpy()
    for k in range(150):
        assert (out[k] == O.ofdm_eq_symbol(x[k], ch[0], k)).all(), k


def test_eq_chain_fixture_host_api(eq):
    csr = np.concatenate([eq["eq_off"], [eq["eq_off"][-1] + eq["eq_nsym"][-1]]]).astype(np.int32)
    pay, info, nok = Z.wifi_rx_eq_batch(eq["eq_sym"], csr, eq["eq_chan"])
    po = eq["eq_payload_off"]
    for i in range(len(eq["eq_crc"])):
        mod, cod, ln = eq["eq_meta"][i]
        assert (info["modulation"][i], info["coding"][i], info["len"][i]) == (mod, cod, ln)
        assert info["crc_ok"][i] == eq["eq_crc"][i], i
        e = eq["eq_payload"][po[i]:po[i + 1]]
        assert (pay[i, :e.size] == e).all(), i
    assert nok == int(eq["eq_crc"].sum())


def test_eq_chain_mixed_vs_oracle(engine, oracle):
    plan = synth.plan_mixed(60, max_len=2300, seed=41)
    sym, off, nsym, meta, chan = synth.packets_time_eq(plan, seed=42, sigma=2.5)
    n = off.size
    engine.reserve(n, int(nsym.max()))
    pay, info = engine.rx(torch.from_numpy(sym).cuda(), torch.from_numpy(off).cuda(),
                          torch.from_numpy(nsym).cuda(), int(nsym.max()),
                          chan=torch.from_numpy(chan).cuda().contiguous())
    pay, info = pay.cpu().numpy(), info.cpu().numpy()
    opay, ores = oracle.rx_batch_time_eq(sym, off, nsym, chan, nthreads=8)
    for i in range(n):
        r = ores[i]
        assert (info[i, 0], info[i, 1], info[i, 2], info[i, 3]) == (r["modulation"], r["coding"], r["len"], r["err"])
        assert info[i, 4] == r["crc_ok"], i
        if not r["err"]:
            L = r["len"] - 4
            assert (pay[i, :L] == opay[i, :L]).all(), i
    assert info[:, 4].sum() > 40


def test_eq_chain_large_54mbps_vs_oracle(engine, oracle):
    """Config-3 shape with a channel: 2048 packets, GPU bit-exact with the oracle."""
    b = txgen.make_batch(2048, seed=77, device="cuda", channel=True, sigma=2.0)
    engine.reserve(2048, b["max_nsym"])
    pay, info = engine.rx(b["sym"], b["sym_off"], b["nsym"], b["max_nsym"], chan=b["chan"])
    pay, info = pay.cpu().numpy(), info.cpu().numpy()
    opay, ores = oracle.rx_batch_time_eq(b["sym"].cpu().numpy(), b["sym_off"].cpu().numpy(),
                                         b["nsym"].cpu().numpy(), b["chan"].cpu().numpy(), nthreads=16)
    assert (info[:, 4] == np.array([r["crc_ok"] for r in ores])).all()
    assert (pay[:, :1500] == opay[:, :1500]).all()
    ok = info[:, 4] == 1
    assert ok.sum() > 1900 and (pay[ok, :1500] == b["payload"][ok]).all()


def test_eq_rejects_missing_coefficients(engine):
    import ctypes as C
    rc = Z.lib().zrx_rx_eq_dev(engine._h, None, None, None, 1, 1, None, None, None)
    assert rc < 0
