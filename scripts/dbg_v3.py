"""Debug helper (GPU): decode one reference frame through k_viterbi3 at several batch
positions and report mismatching bytes against the golden output."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ziria_amd as Z
g = np.load(os.path.join(ROOT, "tests/golden/ref_viterbi.npz"))
cases, so, oo = g["vit_cases"], g["vit_soft_off"], g["vit_out_off"]
for idx in [int(a) for a in sys.argv[1:]] or [9]:
    cr, fl, nz = cases[idx]
    s = g["vit_soft"][so[idx]:so[idx + 1]]
    exp = g["vit_out"][oo[idx]:oo[idx + 1]]
    for pos in (0, 1, 5):
        softs = [s] * (pos + 1)
        offs = np.concatenate([[0], np.cumsum([x.size for x in softs])]).astype(np.int32)
        out, off = Z.viterbi_batch_decode(np.concatenate(softs), offs, np.full(pos + 1, fl, np.int32),
                                          np.full(pos + 1, cr, np.int16))
        got = out[off[pos]:off[pos] + exp.size]
        bad = np.nonzero(got != exp)[0]
        print(f"case {idx} {(int(cr), int(fl), int(nz))} pos {pos}: {bad.size} bad bytes, first {bad[:12].tolist()}")
