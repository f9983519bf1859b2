"""The batched externals over host arrays (include/ziria_rx.h Part 2) through their chunked,
overlapped host pipeline (ziria_amd/csrc/zrx_hostio.hpp): batches large enough to take
several chunks, caller arrays in pageable and in pinned memory, against the device API on
the same inputs (whose parity with the oracle the other GPU tests establish).  Integer work:
bit-exact."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from ziria_amd import txgen  # noqa: E402
from ziria_amd._lib import lib  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402


def _p(a):
    return C.c_void_p(a.data_ptr() if torch.is_tensor(a) else a.ctypes.data)


def _host(a, pinned):
    """numpy (pageable) or a pinned torch CPU tensor holding the same bytes."""
    return torch.from_numpy(np.ascontiguousarray(a)).pin_memory() if pinned else np.ascontiguousarray(a)


def _np(a):
    return a.numpy() if torch.is_tensor(a) else a


@pytest.fixture(scope="module")
def big():
    """5000 config-3 packets (73 MB of symbols: three pipeline chunks) with a few packets cut
    short, decoded once through the device API as the expected result."""
    b = txgen.make_batch(5000, seed=0x51, sigma=4.0, device="cuda")
    nsym = b["nsym"].clone()
    nsym[[7, 2500, 4999]] -= torch.tensor([5, 56, 1], dtype=torch.int32, device="cuda")   # truncated packets
    off = torch.cat([torch.zeros(1, dtype=torch.int64, device="cuda"), torch.cumsum(nsym.to(torch.int64), 0)])
    # pack the (shortened) packets back to back, as a CSR of symbols
    idx = torch.cat([b["sym_off"][i] + torch.arange(int(nsym[i]), device="cuda") for i in range(5000)])
    sym = b["sym"][idx].contiguous()
    e = RxEngine(0)
    e.reserve(5000, b["max_nsym"])
    pay, info = e.rx(sym, off[:-1].contiguous(), nsym, b["max_nsym"])
    torch.cuda.synchronize()
    e.close()
    return dict(sym=sym.cpu().numpy(), csr=off.to(torch.int32).cpu().numpy(), pay=pay.cpu().numpy(),
                info=info.cpu().numpy())


@pytest.mark.parametrize("pin_in,pin_out", [(False, False), (True, True), (True, False), (False, True)])
def test_wifi_rx_batch_chunked(big, pin_in, pin_out):
    n = big["csr"].size - 1
    sym, csr = _host(big["sym"], pin_in), np.ascontiguousarray(big["csr"])
    pay = _host(np.full((n, 4096), 0xA5, np.uint8), pin_out)
    info = _host(np.zeros((n, 8), np.int32), pin_out)
    rc = lib().__ext_wifi_rx_batch(_p(sym), big["sym"].shape[0], _p(csr), n + 1, _p(pay), n * 4096 * 8, _p(info),
                                   n * 8)
    pay, info = _np(pay), _np(info)
    assert rc == int((big["info"][:, 4] == 1).sum()) and rc >= n - 3
    assert (info == big["info"]).all()
    for i in range(n):
        L = max(int(info[i, 2]) - 4, 0) if info[i, 4] else 0
        assert (pay[i, :L] == big["pay"][i, :L]).all(), i
    # bytes past the widest payload a packet of this batch can carry stay the caller's
    assert (pay[:, 1508:] == 0xA5).all()


def _vit_batch(nframes, fl, seed):
    g = np.random.default_rng(seed)
    cr = g.integers(0, 3, nframes).astype(np.int16)
    num, den = {0: (2, 1), 1: (3, 2), 2: (4, 3)}, 48       # coded bits per data bit (CR_12, CR_23, CR_34)
    ns = np.array([-(-(-(-(8 * fl + 6) * num[c][0] // num[c][1])) // den) * den for c in cr], np.int64)
    ns[::7] //= 2                                          # truncated: the decoder stops mid-frame
    ns = (ns // 48 * 48).astype(np.int64)
    so = np.concatenate([[0], np.cumsum(ns)]).astype(np.int32)
    soft = g.integers(0, 8, int(so[-1])).astype(np.int8)
    return soft, so, np.full(nframes, fl, np.int32), cr


@pytest.mark.parametrize("pinned", [False, True])
def test_viterbi_batch_decode_keeps_caller_bytes(pinned):
    """__ext_viterbi_batch_decode scatters only the bytes each frame produced: a frame cut
    short leaves the rest of its output range, and every byte between frames, as the caller
    had them -- the same bytes the device API writes into a pre-filled buffer.  1600 frames of
    1500 bytes: ~58 MB of soft values, two chunks."""
    soft, so, fl, cr = _vit_batch(1600, 1500, 3)
    n = fl.size
    oo = (np.arange(n) * 1600).astype(np.int32)            # 100 caller bytes between frames
    out = _host(np.full(n * 1600, 0x5A, np.uint8), pinned)
    rc = lib().__ext_viterbi_batch_decode(_p(_host(soft, pinned)), soft.size, _p(so), n + 1, _p(fl), n, _p(cr), n,
                                          _p(out), n * 1600 * 8, _p(oo), n)
    assert rc == n
    # the device API over the same frames into a buffer pre-filled the same way
    dev = torch.device("cuda", 0)
    e = RxEngine(0)
    e.reserve(n, 1)
    params = torch.from_numpy(np.stack([fl, cr.astype(np.int32), np.diff(so), np.zeros(n, np.int32)], 1)
                              .astype(np.int32)).to(dev).contiguous()
    d_out = torch.full((n * 1600,), 0x5A, dtype=torch.uint8, device=dev)
    bits = torch.zeros(n, dtype=torch.int32, device=dev)
    e.viterbi(torch.from_numpy(soft).to(dev), torch.from_numpy(so[:-1].astype(np.int64)).to(dev), params, d_out,
              torch.from_numpy(oo.astype(np.int64)).to(dev), bits)
    torch.cuda.synchronize()
    e.close()
    assert (_np(out) == d_out.cpu().numpy()).all()
    b = bits.cpu().numpy()
    assert (b[::7] < 8 * 1500).all() and (b[1::7] == 8 * 1500).all()


def test_wifi_rx_eq_batch_chunked():
    """The EQ external (ChannelEqualization + PilotTrack) through the same pipeline: 4600
    packets through a channel (three chunks, the channel coefficients uploaded with their
    chunk's symbols), pageable arrays, against the device API."""
    b = txgen.make_batch(4600, seed=0x52, sigma=2.0, device="cuda", channel=True)
    n, S = 4600, b["max_nsym"]
    e = RxEngine(0)
    e.reserve(n, S)
    pay_d, info_d = e.rx(b["sym"], b["sym_off"], b["nsym"], S, chan=b["chan"])
    torch.cuda.synchronize()
    e.close()
    pay_d, info_d = pay_d.cpu().numpy(), info_d.cpu().numpy()
    sym = np.ascontiguousarray(b["sym"].cpu().numpy())
    chan = np.ascontiguousarray(b["chan"].cpu().numpy())
    csr = (np.arange(n + 1) * S).astype(np.int32)
    pay = np.zeros((n, 4096), np.uint8)
    info = np.zeros((n, 8), np.int32)
    rc = lib().__ext_wifi_rx_eq_batch(_p(sym), sym.shape[0], _p(csr), n + 1, _p(chan), n * 64, _p(pay), n * 4096 * 8,
                                      _p(info), n * 8)
    assert rc == int((info_d[:, 4] == 1).sum()) > n - 50
    assert (info == info_d).all()
    ok = info[:, 4] == 1
    assert (pay[ok, :1500] == pay_d[ok, :1500]).all() and (pay[ok, :1500] == b["payload"][ok]).all()


@pytest.mark.parametrize("shards", [1, 3])
def test_wifi_rx_batch_chunked_mixed(shards):
    """A mixed batch through the chunked pipeline: 3000 distinct config-5 packets
    (8 MCS, PSDU 64..4095 B; ~110 MB of symbols: several chunks whose widest payload `cw` and
    longest packet differ chunk to chunk, the split plan's hint read across chunks), pageable
    arrays, on one and on three shards of GPU 0, against the device API on the same packets."""
    import ziria_amd as Z
    m = txgen.make_mixed_fast(3000, min_len=64, max_len=4095, sigma=3.0, seed=0xC4C4, device="cuda")
    n, S = 3000, m["max_nsym"]
    e = RxEngine(0)
    e.reserve(n, S)
    pay_d, info_d = e.rx(m["sym"], m["sym_off"], m["nsym"], S)
    torch.cuda.synchronize()
    e.close()
    pay_d, info_d = pay_d.cpu().numpy(), info_d.cpu().numpy()
    off, ns = m["sym_off"].cpu().numpy(), m["nsym"].cpu().numpy()
    sym = m["sym"].cpu().numpy()
    idx = np.concatenate([np.arange(o, o + k) for o, k in zip(off, ns)])
    sym = np.ascontiguousarray(sym[idx])
    csr = np.concatenate([[0], np.cumsum(ns)]).astype(np.int32)
    assert sym.nbytes > 3 * (32 << 20)                      # (more than three chunks)
    pay = np.full((n, 4096), 0xA5, np.uint8)
    info = np.zeros((n, 8), np.int32)
    try:
        if shards > 1:
            Z.set_devices([0] * shards, 0)
        rc = lib().__ext_wifi_rx_batch(_p(sym), sym.shape[0], _p(csr), n + 1, _p(pay), n * 4096 * 8, _p(info), n * 8)
        assert Z.node_stats()["last_shards"] == shards
    finally:
        Z.set_devices(None, -1)
    assert rc == int((info_d[:, 4] == 1).sum()) > n // 3
    assert (info == info_d).all()
    for i in range(n):
        L = max(int(info[i, 2]) - 4, 0) if info[i, 4] else 0
        assert (pay[i, :L] == pay_d[i, :L]).all(), i
