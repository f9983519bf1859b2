"""Offline model of k_viterbi3's schedule on MI355X: rows -> waves -> blocks -> CUs/SIMDs.

Used to compare Viterbi row plans for mixed batches (BASELINE config 5) before spending GPU
time on them.  Model:
  * 256 CUs x 4 SIMDs; a block is 4 waves (one per SIMD of its CU), at most 4 blocks per CU
    (LDS ring); blocks 0..1023 start on CU b mod 256, later blocks take the first CU slot
    that frees (the dispatcher, scripts/ubench/hwid.hip);
  * a wave runs one pass per code rate among its 4 rows, each as long as its longest row;
  * a SIMD with k active waves runs S(k) wave-columns per second in total, shared equally
    (S(1) from config 2 at one wave per SIMD, S(4) from config 3; S(2), S(3) interpolated).
Plans: 'cur' (k_pkt_plan as built: segment length 11/8 L, (rate, length) sort, snake), and
'chain' (rows packed from frames and segments of one rate up to a target length, one round).
"""
import argparse
import heapq
import math

import numpy as np

NCBPS = {0: 48, 1: 96, 2: 192, 3: 288}
MCS8 = [(0, 0), (0, 2), (1, 0), (1, 2), (2, 0), (2, 2), (3, 1), (3, 2)]
S_K = {1: 21.7e6, 2: 31.0e6, 3: 36.0e6, 4: 38.6e6}
NCU = 256


def ndbps(mod, cod):
    nc = NCBPS[mod]
    return nc // 2 if cod == 0 else (nc * 2 // 3 if cod == 1 else nc * 3 // 4)


def config5(seed=0x3C5, n=16384, min_len=64, max_len=4095):
    rng = np.random.default_rng(seed)
    mcs = rng.integers(0, 8, n)
    lens = rng.integers(min_len, max_len + 1, n)
    pk = []
    for m, L in zip(mcs, lens):
        if L > 2048:
            continue                                   # header error: no trellis row
        mod, cod = MCS8[m]
        nd = ndbps(mod, cod)
        nsym = (16 + 8 * (int(L) - 4) + 32 + 6 + nd - 1) // nd
        soft = nsym * NCBPS[mod]
        cols = soft // 2 if cod == 0 else ((soft // 3) * 2 if cod == 1 else (soft // 4) * 3)
        E = 8 * (int(L) + 2) + 6
        pk.append((cod, min(cols, E + 30), E, cols))
    return pk


def uniform(fl, cr, n):
    E = 8 * fl + 6
    return [(cr, E, E, E + 72)] * n


def udiv_small(y, n):
    return y if n <= 1 else y // n


def seg_start(E, nseg, k):
    return 0 if k == 0 else 768 * udiv_small((2 * k * E + nseg * 768) // 1536, nseg)


def seg_count(E, cols, L):
    if cols < E or E < 3072 or L == 0:
        return 1
    n = (cols + L - 1) // L
    n = min(n, E // 1536)
    return min(max(n, 1), 8)


def segments(E, cols, nseg):
    out = []
    for k in range(nseg):
        S = seg_start(E, nseg, k)
        stop = seg_start(E, nseg, k + 1) + 256 + 30 if k + 1 < nseg else cols
        out.append(min(stop, E + 30) - S)
    return out


def order_place(pos, nfull, ncu=NCU):
    b = pos >> 4
    if b >= nfull:
        return pos
    r, c = divmod(b, ncu)
    base = r * ncu
    m = min(ncu, nfull - base)
    return ((base + m - 1 - c) if r & 1 else b) * 16 + (pos & 15)


def plan_cur(pk, num=11, uniform_batch=False):
    tcols = sum(c for _, _, _, c in pk)
    L = max(1536, -(-tcols // (64 * NCU)))
    Lm = (L + L // 8) if uniform_batch else max(L * num // 8, 1536)
    rows = []
    keyed = []
    for cr, run, E, cols in pk:
        n = seg_count(E, cols, Lm)
        ln = cols if n <= 1 else -(-cols // n) + 286
        bodies = min((ln + 23) // 24, 1023)
        keyed.append(((cr, -bodies), [(cr, s) for s in (segments(E, cols, n) if n > 1 else [run])]))
    keyed.sort(key=lambda x: x[0])
    flat = [r for _, rs in keyed for r in rs]
    nfull = len(flat) >> 4
    placed = [None] * len(flat)
    for i, r in enumerate(flat):
        placed[order_place(i, nfull)] = r
    return [[r] for r in placed]                     # one item per row


def plan_chain(pk, rows_target=64 * NCU, over=1.0, seg_num=8):
    """Rows of one rate, each a chain of frames/segments up to ~target columns, one round."""
    tcols = sum(c for _, _, _, c in pk)
    T = max(1536, int(over * tcols / rows_target))
    items = {0: [], 1: [], 2: []}
    for cr, run, E, cols in pk:
        n = seg_count(E, cols, T * seg_num // 8)
        for s in (segments(E, cols, n) if n > 1 else [run]):
            items[cr].append(s)
    rows = []
    for cr in (0, 1, 2):
        its = sorted(items[cr], reverse=True)
        nrow = max(1, round(sum(its) / T))
        heap = [(0, i) for i in range(nrow)]
        rr = [[] for _ in range(nrow)]
        for s in its:                                  # LPT: longest item onto the least-loaded row
            load, i = heapq.heappop(heap)
            rr[i].append((cr, s))
            heapq.heappush(heap, (load + s + 24, i))
        rr.sort(key=lambda r: -sum(s for _, s in r))
        rows += rr
    return rows


def simulate(rows, verbose=False):
    """rows: list of rows, each a list of (rate, columns) items run back to back. Returns seconds."""
    # pad to whole waves
    while len(rows) % 4:
        rows.append([])
    waves = []
    for w in range(0, len(rows), 4):
        q = rows[w:w + 4]
        # the wave runs item after item per row in lockstep passes per rate: approximate as the
        # longest row's total plus one pass per extra rate in the wave
        tot = max((sum(s for _, s in r) for r in q), default=0)
        rates = {cr for r in q for cr, _ in r}
        if len(rates) > 1:
            tot = sum(max((sum(s for c2, s in r if c2 == cr) for r in q), default=0) for cr in rates)
        waves.append(tot + 300 if tot else 0)          # + tail (final traceback, launch)
    blocks = [waves[i:i + 4] + [0] * (4 - len(waves[i:i + 4])) for i in range(0, len(waves), 4)]
    # event simulation: SIMDs hold (remaining) work of active waves
    simd = [[] for _ in range(NCU * 4)]                 # per SIMD: list of [remaining, block id]
    block_left = {}
    free_slots = []                                     # CUs with a free block slot (time order)
    t = 0.0
    nb = len(blocks)
    nxt = 0
    cu_blocks = [0] * NCU

    def place(b, cu):
        block_left[b] = 0
        for j, wl in enumerate(blocks[b]):
            if wl > 0:
                simd[cu * 4 + j].append([float(wl), b])
                block_left[b] += 1
        cu_blocks[cu] += 1
        if block_left[b] == 0:
            cu_blocks[cu] -= 1
            return False
        return True

    while nxt < nb and nxt < 4 * NCU:
        place(nxt, nxt % NCU)
        nxt += 1
    block_cu = {b: b % NCU for b in range(min(nb, 4 * NCU))}
    done_t = 0.0
    while True:
        # next completion time
        best = math.inf
        for i, ws in enumerate(simd):
            if ws:
                r = S_K[min(len(ws), 4)] / len(ws)
                m = min(w[0] for w in ws)
                best = min(best, m / r)
        if best == math.inf:
            break
        t += best
        finished_blocks = []
        for i, ws in enumerate(simd):
            if ws:
                r = S_K[min(len(ws), 4)] / len(ws)
                for w in ws:
                    w[0] -= best * r
                keep = []
                for w in ws:
                    if w[0] <= 1e-6:
                        block_left[w[1]] -= 1
                        if block_left[w[1]] == 0:
                            finished_blocks.append(w[1])
                    else:
                        keep.append(w)
                simd[i] = keep
        for b in finished_blocks:
            cu = block_cu[b]
            cu_blocks[cu] -= 1
            while nxt < nb:
                block_cu[nxt] = cu
                ok = place(nxt, cu)
                nxt += 1
                if ok:
                    break
        done_t = t
    return done_t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="c5")
    a = ap.parse_args()
    if a.what == "probe":
        for fl in (512, 1024, 1500, 2048):
            E = 8 * fl + 6
            n = int(150e6 // (-(-E // 72) * 72))
            pk = uniform(fl, 0, n)
            rows = plan_cur(pk, uniform_batch=True)
            t = simulate(rows)
            print(f"uniform fl {fl}: {len(rows)} rows, {n * E / t / 1e9:.1f} G col/s")
        return
    pk = config5()
    tc = sum(c for _, _, _, c in pk)
    print(f"config 5: {len(pk)} frames, {tc / 1e6:.2f} M columns")
    rows = plan_cur(pk)
    t = simulate(rows)
    print(f"cur: {len(rows)} rows, {t * 1e3:.3f} ms, {tc / t / 1e9:.1f} G col/s")
    for over in (0.95, 1.0, 1.05):
        for sn in (8, 12, 16):
            rows = plan_chain(pk, over=over, seg_num=sn)
            t = simulate(rows)
            print(f"chain over {over} seg {sn}/8: {len(rows)} rows, {t * 1e3:.3f} ms, {tc / t / 1e9:.1f} G col/s")


if __name__ == "__main__":
    main()
