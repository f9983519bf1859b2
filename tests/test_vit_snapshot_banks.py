"""The LDS bank pattern of k_viterbi3's snapshot stores (zrx_viterbi3.hpp Packet::snapshot),
restated on the host: which byte each lane writes for every (snapshot k, dword d, half h)
store, banked as the guide's LDS model banks a ds_write (MI355X_MICROARCH.md §LDS: 32 banks
of 4 bytes, lane groups 0-31 and 32-63, one extra cycle per extra distinct dword on a busy
bank).  Every store instruction is exactly 2-way conflicted (rows r and r + 2 of a lane group
are 32 dwords apart), which accounts for the SQ_LDS_BANK_CONFLICT count of the PMC summary
(DESIGN.md §5 round 5); a 2-way ds_write conflict costs no time in that model."""
import json
import os

from tests import vit8_model as V8

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rotl6(x, k):
    return x & 63 if k == 0 else ((x << k) | (x >> (6 - k))) & 63


def rev6(x):
    return int(format(x, "06b")[::-1], 2)


def snap_delta(k, d, h):
    """v3::snap_delta: ring-index offset of in-lane position bits (d, h) at snapshot k"""
    p = h | (d << 1)
    o = 0
    for b in range(3):
        if (p >> b) & 1:
            o |= 1 << (5 - (b + 2 * k) % 6)
    return o


def extra_cycles(addrs):
    tot = 0
    for group in (range(0, 32), range(32, 64)):
        banks = {}
        for lane in group:
            banks.setdefault((addrs[lane] // 4) % 32, set()).add(addrs[lane] // 4)
        tot += max(len(v) for v in banks.values()) - 1
    return tot


def store_instructions():
    """(name, byte address per lane) of one wave's snapshot stores in a 24-column body: k = 0, 1
    as 8 byte stores (d, h), k = 2 as 2 dword stores of consecutive ring bytes."""
    rows = [(lane // 8, lane % 8) for lane in range(64)]              # (row in wave, lane in row)
    for k in (0, 1):
        for d in range(4):
            for h in range(2):
                yield (k, d, h), [r * 64 + rev6(rotl6(V8.pos_of(l, 0, 0), 2 * k)) + snap_delta(k, d, h) for r, l in rows]
    for e in range(2):
        yield (2, 2 * e, 0), [r * 64 + rev6(rotl6(V8.pos_of(l, 0, 0), 4)) + snap_delta(2, 2 * e, 0) for r, l in rows]


def test_positions_cover_the_ring_line():
    """Over a snapshot's stores every lane of a row writes distinct bytes and the row's stores
    together write all 64 bytes of its ring line (k = 2: its dword stores cover 4 bytes each)."""
    for k in (0, 1, 2):
        written = set()
        for (kk, d, h), addrs in store_instructions():
            if kk != k:
                continue
            row0 = addrs[:8]
            assert len(set(row0)) == 8
            for a in row0:
                written.update(range(a, a + (4 if k == 2 else 1)))
        assert written == set(range(64)), k


def test_every_store_is_two_way():
    counts = [extra_cycles(addrs) for _, addrs in store_instructions()]
    assert counts == [2] * 18


def test_accounts_for_the_pmc_count():
    per_body = sum(extra_cycles(addrs) for _, addrs in store_instructions())    # one wave
    waves, bodies = 16384 // 8, -(-(8 * 1506 + 6) // 24)                       # config 3: 2048 waves x 503 bodies
    model = per_body * waves * bodies
    s = json.load(open(os.path.join(ROOT, "profiles", "pmc_summary.json")))
    measured = s["kernels"]["k_viterbi3"]["counters"]["SQ_LDS_BANK_CONFLICT"]
    assert abs(measured - model) / measured < 0.05, (model, measured)
