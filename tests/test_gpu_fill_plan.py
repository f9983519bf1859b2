"""The packed plan of a mixed batch (zrx_kernels.hip plan_waves_fill, k_viterbi3's packed rows),
read back through zrx_plan_dump after a real rx-chain launch on a BASELINE config-5 batch:
every decodable frame is covered once by its segments in order, in one row of its waves; the
seams obey the table geometry's rules (window starts, 256 <= J, J + 64 <= E, at most 7); a
wave's items share a rate; the 8 items of a part share their segment index and seam, so the
rows' traceback windows fall on the same columns; and the waves are balanced.  Decoding through this plan is checked bit-exact
elsewhere (test_gpu_fullsize.py::test_fullsize_config5_vs_port and the mixed chain tests)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from ziria_amd import txgen  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402


def _piece(k, n, J, cols):
    """columns [start, stop) of segment k of n (table geometry: S_k = 24 floor((J_k - 256) / 24),
    a segment runs to J_{k+1} + 30)"""
    start = 0 if k == 0 else (J[k - 1] - 256) // 24 * 24
    stop = J[k] + 30 if k + 1 < n else cols
    return start, stop


@pytest.mark.parametrize("npkts", [16384, 3000])
def test_fill_plan_invariants(npkts):
    m = txgen.make_mixed_fast(npkts, min_len=64, max_len=4095, sigma=3.0, seed=0xF111 + npkts, device="cuda")
    e = RxEngine(0)
    e.reserve(npkts, m["max_nsym"])
    pay, info = e.rx(m["sym"], m["sym_off"], m["nsym"], m["max_nsym"])
    torch.cuda.synchronize()
    d = e.plan_dump(npkts)
    e.close()
    h = d["header"]
    assert h[6] == 1 and h[2] == 0 and h[5] == 0, h          # packed, not uniform, nothing dropped
    assert h[0] % 8 == 0
    nw = int(h[0]) // 8
    wfirst = d["wfirst"][:nw + 1]
    assert wfirst[0] == 0 and (np.diff(wfirst) >= 0).all()
    items = d["items"][:8 * wfirst[nw]]
    mod, cod, plen = m["meta"][:, 0], m["meta"][:, 1], m["meta"][:, 2]
    decodable = plen <= 2048
    cols = np.array([txgen.n_data_symbols(int(a), int(b), int(L) - 4) * txgen.ndbps(int(a), int(b))
                     for a, b, L in zip(mod, cod, plen)])
    E = 8 * (plen + 2) + 6                                   # (the Viterbi frame: SERVICE + PSDU, Decode.blk:59)
    seen = {}
    wave_len = np.zeros(nw, np.int64)
    for w in range(nw):
        rate = 0 if w < h[14] else 1 if w < h[15] else 2
        for i in range(wfirst[w], wfirst[w + 1]):
            part_len, ks, Js = 0, set(), set()
            for j in range(8):
                p, kn = int(items[8 * i + j, 0]), int(items[8 * i + j, 1])
                if p < 0:
                    continue
                k, n = kn & 0xFF, (kn >> 8) & 0xFF
                assert n == d["segs"][p] and 0 <= k < n <= 8 and int(cod[p]) == rate
                seen.setdefault(p, []).append((k, i, j))
                J = [256 * int(c) for c in d["cuts"][p, :n - 1]]
                a, b = _piece(k, n, J, int(cols[p]))
                assert a < b
                part_len = max(part_len, b - a)
                ks.add(k)
                if k:
                    Js.add(J[k - 1])
            # a part's rows start together at one segment index and seam: their windows align
            assert len(ks) == 1 and len(Js) <= 1, (w, i, ks, Js)
            wave_len[w] += part_len
    assert set(seen) == set(np.nonzero(decodable)[0].tolist())
    for p, lst in seen.items():
        n = int(d["segs"][p])
        assert [k for k, _, _ in lst] == list(range(n)), (p, lst)
        assert len({j for _, _, j in lst}) == 1                   # one row of its waves
        assert all(lst[x][1] < lst[x + 1][1] for x in range(n - 1))   # segments in part order
        J = [256 * int(c) for c in d["cuts"][p, :n - 1]]
        assert all(256 <= x and x + 64 <= E[p] for x in J) and J == sorted(set(J)), (p, J)
    used = wave_len[wave_len > 0]
    mean = used.mean()
    print(f"waves {nw}, parts {wfirst[nw]}, wave columns mean {mean:.0f} max {used.max()}")
    if npkts == 16384:                                       # one block round; balanced to a few windows
        assert nw <= 8 * 256 + 2 and used.max() <= mean + 1000
    assert (info[:, 4].cpu().numpy()[decodable] == 1).mean() > 0.95
