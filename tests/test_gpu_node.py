"""The batched externals split over the node's logical shards (zrx_set_devices,
ziria_amd/csrc/zrx_shard.hpp), on the GPU: two and three shards forced onto device 0 run the
very code path an 8-GPU node takes (one context, stream, copy streams and host thread per
shard, contiguous packet ranges, outputs written straight into the caller's arrays), checked
bit-exactly against the reference-pinned fixtures, the oracle and, at BASELINE config 3's
full 16384 packets, the host port.  Also the page-locking of recurring caller arrays
(zrx_set_host_register).  Integer/byte work: bit-exact."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import ziria_amd as Z  # noqa: E402
from ziria_amd import txgen  # noqa: E402
from tests import fe_cases  # noqa: E402


@pytest.fixture
def shards(request):
    """zrx_set_devices([0] * k, min_shard_bytes=0): every call spread over k shards on GPU 0;
    the default node (and host-register mode) restored afterwards."""
    def use(k):
        Z.set_devices([0] * k, 0)
        assert Z.get_devices() == [0] * k
    yield use
    Z.set_devices(None, -1)
    Z.set_host_register(1)


def _threads():
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return 8


@pytest.mark.parametrize("k", [2, 3])
@pytest.mark.parametrize("tag", ["c54", "mix"])
def test_sharded_chain_reference_packets(golden, shards, k, tag):
    shards(k)
    g = golden["ref_chain"]
    sym, off, nsym = g[f"{tag}_sym"], g[f"{tag}_off"], g[f"{tag}_nsym"]
    csr = np.concatenate([off, [off[-1] + nsym[-1]]]).astype(np.int32)
    pay, info, nok = Z.wifi_rx_batch(sym, csr)
    assert Z.node_stats()["last_shards"] == min(k, csr.size - 1)
    po, crc, meta = g[f"{tag}_payload_off"], g[f"{tag}_crc"], g[f"{tag}_meta"]
    for i in range(len(crc)):
        assert (info["modulation"][i], info["coding"][i], info["len"][i]) == tuple(meta[i])
        assert info["crc_ok"][i] == crc[i], i
        e = g[f"{tag}_payload"][po[i]:po[i + 1]]
        assert (pay[i, :e.size] == e).all(), i
    assert nok == int(crc.sum())


def test_sharded_chain_mixed_vs_oracle(shards, oracle):
    """Mixed rates and lengths (unequal shards by bytes) through three shards vs the oracle."""
    shards(3)
    m = txgen.make_mixed(96, max_len=2200, sigma=3.0, seed=5, device="cuda")
    sym, off, ns = m["sym"].cpu().numpy(), m["sym_off"].cpu().numpy(), m["nsym"].cpu().numpy()
    # the externals take a CSR of symbols: repack the packets back to back
    idx = np.concatenate([np.arange(o, o + n) for o, n in zip(off, ns)])
    csr = np.concatenate([[0], np.cumsum(ns)]).astype(np.int32)
    pay, info, nok = Z.wifi_rx_batch(sym[idx], csr)
    assert Z.node_stats()["last_shards"] == 3
    opay, ores = oracle.rx_batch_time(sym, off, ns, nthreads=8)
    for i, r in enumerate(ores):
        assert (info["modulation"][i], info["coding"][i], info["len"][i], info["header_err"][i]) == \
            (r["modulation"], r["coding"], r["len"], r["err"]), i
        if r["err"]:
            continue
        assert info["crc_ok"][i] == r["crc_ok"], i
        L = r["len"] - 4
        assert (pay[i, :L] == opay[i, :L]).all(), i
    assert nok == sum(r["crc_ok"] for r in ores if not r["err"])


def test_sharded_fullsize_config3_vs_port(shards, oracle):
    """BASELINE config 3 at full size, 16384 packets (239 MB of samples in pageable host memory),
    through __ext_wifi_rx_batch split over three shards: every packet against the host port
    and the transmitted payload."""
    shards(3)
    b = txgen.make_batch(16384, seed=0x5EED, sigma=4.0, device="cuda")
    S = b["max_nsym"]
    sym = np.ascontiguousarray(b["sym"].cpu().numpy())
    csr = (np.arange(16385) * S).astype(np.int32)
    pay, info, nok = Z.wifi_rx_batch(sym, csr)
    assert Z.node_stats()["last_shards"] == 3
    opay, res = oracle.rx_batch_time_fast(sym, b["sym_off"].cpu().numpy(), b["nsym"].cpu().numpy(),
                                          nthreads=_threads())
    assert nok == 16384 and all(r["crc_ok"] for r in res)
    assert (info["crc_ok"] == 1).all() and (info["len"] == 1504).all()
    assert (pay[:, :1500] == opay[:, :1500]).all()
    assert (pay[:, :1500] == b["payload"]).all()


def test_sharded_viterbi_vs_oracle(shards, oracle):
    shards(3)
    from tests.golden import synth
    rng = np.random.default_rng(77)
    softs, offs, fls, crs = [], [0], [], []
    for i in range(67):
        cr = int(rng.integers(0, 3))
        fl = int(rng.integers(1, 700))
        s = synth.viterbi_soft(cr, fl, int(rng.integers(-1, 5)), seed=1000 + i)
        if i % 5 == 0:
            s = s[: max(48, (s.size // 2) // 48 * 48)]
        softs.append(s); offs.append(offs[-1] + s.size); fls.append(fl); crs.append(cr)
    soft = np.concatenate(softs)
    # outputs in reverse packet order with gaps: each shard scatters into its own ranges
    fl_a = np.array(fls, np.int32)
    oo = np.zeros(len(fls), np.int32)
    pos = 0
    for i in reversed(range(len(fls))):
        oo[i] = pos
        pos += fls[i] + 5
    out, off = Z.viterbi_batch_decode(soft, np.array(offs, np.int32), fl_a, np.array(crs, np.int16), oo)
    assert Z.node_stats()["last_shards"] == 3
    for i in range(len(fls)):
        exp = oracle.viterbi_decode(soft[offs[i]:offs[i + 1]], fls[i], crs[i])
        assert (out[off[i]:off[i] + exp.size] == exp).all(), i


def test_viterbi_overlapping_outputs_rejected():
    soft = np.zeros(96, np.int8)
    so = np.array([0, 48, 96], np.int32)
    with pytest.raises(Z.ZiriaRxError):
        Z.viterbi_batch_decode(soft, so, np.array([10, 10], np.int32), np.zeros(2, np.int16),
                               np.array([0, 9], np.int32))
    out, _ = Z.viterbi_batch_decode(soft, so, np.array([10, 10], np.int32), np.zeros(2, np.int16),
                                    np.array([0, 10], np.int32))             # adjacent: fine
    assert out.size >= 20


def test_sharded_fft64_eq_stream_tx(golden, shards, oracle):
    """The other batched externals through three shards: FFT64 (reference vectors), the EQ
    chain (reference-pinned fixture), receiver() over captures (the reference's end-to-end KATs
    plus oracle-checked variants) and the TX chain (oracle)."""
    shards(3)
    g = golden["ref_fft64"]
    assert (Z.sora_fft64_batch(g["fft_in"]) == g["fft_out"]).all()
    eq = golden["ref_eq"]
    csr = np.concatenate([eq["eq_off"], [eq["eq_off"][-1] + eq["eq_nsym"][-1]]]).astype(np.int32)
    pay, info, nok = Z.wifi_rx_eq_batch(eq["eq_sym"], csr, eq["eq_chan"])
    po = eq["eq_payload_off"]
    for i in range(len(eq["eq_crc"])):
        assert info["crc_ok"][i] == eq["eq_crc"][i], i
        e = eq["eq_payload"][po[i]:po[i + 1]]
        assert (pay[i, :e.size] == e).all(), i
    assert nok == int(eq["eq_crc"].sum())
    fe = golden["ref_fe"]
    rx, real = fe_cases.kat_streams(fe)
    caps = [real] + fe_cases.variants(fe, 20, seed=23) + [real]
    off = np.cumsum([0] + [c.shape[0] for c in caps]).astype(np.int32)
    pay, info, det, nok = Z.wifi_rx_stream_batch(np.concatenate(caps), off)
    assert Z.node_stats()["last_shards"] == 3
    for i in (0, len(caps) - 1):
        assert det[i, 0] == 1 and info["crc_ok"][i] == 1
        assert (pay[i, :fe["real_out"].size] == fe["real_out"]).all()
    for i, c in enumerate(caps[1:-1], 1):
        opay, r, odet, _, _ = oracle.rx_stream(c)
        assert det[i, 0] == (r["ret"] != -1), i
        if r["ret"] == 0:
            assert info["crc_ok"][i] == r["crc_ok"], i
            L = max(r["len"] - 4, 0)
            assert (pay[i, :L] == opay[:L]).all(), i
    rng = np.random.default_rng(3)
    pk = []
    for i in range(24):
        mod, cod = [(0, 0), (0, 2), (1, 0), (1, 2), (2, 0), (2, 2), (3, 1), (3, 2)][i % 8]
        ln = int(rng.integers(4, 2049))
        pk.append(np.concatenate([oracle.plcp_header(mod, cod, ln), rng.integers(0, 256, ln - 4).astype(np.uint8)]))
    out, toff = Z.wifi_tx_batch(pk)
    assert Z.node_stats()["last_shards"] == 3
    for i, p in enumerate(pk):
        exp = oracle.tx_packet(p)
        assert (out[toff[i]:toff[i + 1]] == exp).all(), i


def test_host_register_reused_and_modified_arrays(shards):
    """Mode 2: the same pageable arrays handed back call after call are page-locked once and
    copied in place from then on; rewriting their contents between calls is seen by the next
    call (bit-exact against the device API's result for each content); mode 0 releases them."""
    shards(2)
    Z.set_host_register(2)
    n = 2000
    bs = [txgen.make_batch(n, seed=0x600 + j, sigma=4.0, device="cuda") for j in range(2)]
    S = bs[0]["max_nsym"]
    csr = (np.arange(n + 1) * S).astype(np.int32)
    sym = np.ascontiguousarray(bs[0]["sym"].cpu().numpy())
    pay = np.full((n, 4096), 0xA5, np.uint8)
    info = np.zeros((n, 8), np.int32)
    import ctypes as C
    P = lambda a: a.ctypes.data_as(C.c_void_p)
    call = lambda: Z.lib().__ext_wifi_rx_batch(P(sym), sym.shape[0], P(csr), n + 1, P(pay), n * 4096 * 8, P(info),
                                               n * 8)
    st0 = Z.node_stats()
    assert call() == n and (pay[:, :1500] == bs[0]["payload"]).all()
    st1 = Z.node_stats()
    assert st1["register_mode"] == 2 and st1["registrations"] - st0["registrations"] == 3   # sym, payload, info
    assert call() == n
    st2 = Z.node_stats()
    assert st2["registrations"] == st1["registrations"] and st2["register_hits"] - st1["register_hits"] == 3
    sym[:] = bs[1]["sym"].cpu().numpy()                            # new contents, same arrays
    assert call() == n and (pay[:, :1500] == bs[1]["payload"]).all() and (info[:, 4] == 1).all()
    sym[5 * S] = 0                                                 # packet 5's SIGNAL symbol wiped
    assert call() == n - 1 and info[5, 4] == 0
    Z.set_host_register(0)
    assert Z.node_stats()["registered_ranges"] == 0
    assert call() == n - 1 and (pay[:5, :1500] == bs[1]["payload"][:5]).all()
