"""Host restatement of k_descramble_crc's LDS index arithmetic (zrx_kernels.hip, "descramble +
CRC"): the XOR-swizzled payload copy and the keystream table indexed by 32 x byte offset.

For every payload length the kernel admits (len <= 2048, parsePLCPHeader.blk:171-174, so
plen = len - 4 <= 2044) the positions the stores write and the ds_read_b128 chunk loads read
must give every lane the payload words of its 32-byte chunk of the right-aligned 2048-byte
frame (zeros before the payload), and no two stored words may share a position.  For every
scrambler phase the remapped keystream word must be the byte-offset table's word.
"""
import numpy as np

GUARD, REGION = 16, 544


def pos(v):
    return v ^ (((v >> 6) & 1) << 2)


def chunk_words(plen):
    """The 9 words lane L reads, as payload word indices (-1 = a zero word), per lane."""
    c = (plen - 2048) >> 2
    u = (-c) & 7
    lds = np.full(REGION, -2, dtype=np.int64)       # -2: never written (stale)
    lds[:GUARD] = -1
    for lane in range(8):                           # per-packet zeros, v 16..23
        lds[pos(GUARD + lane)] = -1
    v0 = np.arange(64) + GUARD + u
    pe = pos(v0)
    po = pe ^ 4
    for k in range(8):
        i = np.arange(64) + 64 * k
        p = (po if k & 1 else pe) + 64 * k
        assert p.max() < REGION
        assert np.array_equal(p, pos(v0 + 64 * k))
        # a word past the payload is stored as zero (masked); keep its index to check coverage
        lds[p] = np.where(4 * i < plen, i, -1)
    out = np.zeros((64, 9), dtype=np.int64)
    vl = np.maximum(8 * np.arange(64) + GUARD + c + u, 0)
    assert np.all(vl % 8 == 0)
    p0 = pos(vl)
    assert np.all(p0 % 4 == 0)                      # 16-byte aligned ds_read_b128
    for j in range(4):
        out[:, j] = lds[p0 + j]
        out[:, 4 + j] = lds[(p0 ^ 4) + j]
    last = lds[pos(528 + c + u)]
    out[:63, 8] = out[1:, 0]                        # wave_shl:1 of word 0
    out[63, 8] = last
    return out


def test_payload_copy_chunks_all_lengths():
    for plen in range(4, 2045):
        got = chunk_words(plen)
        assert (got != -2).all(), plen               # nothing stale is read
        c = (plen - 2048) >> 2
        want = 8 * np.arange(64)[:, None] + c + np.arange(9)[None, :]
        want = np.where((want >= 0) & (4 * want < plen), want, -1)
        assert np.array_equal(got, want), plen


def test_payload_copy_positions_distinct():
    for u in range(8):
        v = GUARD + u + np.arange(512)
        p = pos(v)
        assert len(set(p.tolist())) == 512 and p.max() < REGION and p.min() >= GUARD


def test_chunk_loads_conflict_free():
    # ds_read_b128 lane groups (MI355X_MICROARCH.md, LDS): 16 lanes on 64 banks of 4 bytes
    groups = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
              list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
    groups += [[l + 32 for l in g] for g in groups]
    for plen in (4, 100, 1496, 1500, 2044):
        c = (plen - 2048) >> 2
        u = (-c) & 7
        vl = 8 * np.arange(64) + GUARD + c + u
        for half in (0, 4):
            p = pos(vl) ^ half
            for g in groups:
                if (vl[g] < 0).any():
                    continue                        # clamped lanes share one address (broadcast)
                banks = {(int(p[l]) // 4) % 16 for l in g}
                assert len(banks) == 16, (plen, g)


def test_keystream_remap():
    rng = np.random.default_rng(1)
    kscrw = rng.integers(0, 2**32, 127, dtype=np.uint64)   # any 127-periodic word table
    scrw4 = kscrw[(4 * np.arange(320)) % 127]
    for phase in range(127):
        n0 = (16 * phase) % 127
        base = (4 * phase) % 127
        for k in range(8):
            i = np.arange(64) + 64 * k
            j = base + np.arange(64) + (k >> 1) + 64 * (k & 1)
            assert j.max() < 320
            assert np.array_equal(scrw4[j], kscrw[(n0 + 4 * i) % 127])
        for plen in (0, 1, 5, 1496, 2044):
            assert scrw4[(32 * (n0 + plen)) % 127] == kscrw[(n0 + plen) % 127]
