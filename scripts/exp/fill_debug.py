"""Debug probe for the packed plan: one config-5 batch decoded with the packed plan and with
rows of whole frames (ZRX_FILL=0 in a child), decoded bytes compared per packet; the failing
packets' items located in the plan (row, position in the row, segment)."""
import os
import subprocess
import sys

import numpy as np

sys.path.insert(0, ".")
mode = sys.argv[1] if len(sys.argv) > 1 else "main"
if mode == "main":
    r = subprocess.run([sys.executable, __file__, "dec"], env=dict(os.environ, ZRX_FILL="0"))
    assert r.returncode == 0
import torch  # noqa: E402
from ziria_amd import txgen  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402

dev = torch.device("cuda", 0)
m = txgen.make_mixed_fast(16384, min_len=64, max_len=4095, sigma=3.0, seed=0xF111 + 16384, device=dev)
e = RxEngine(0)
e.reserve(16384, m["max_nsym"])
pay, info = e.rx(m["sym"], m["sym_off"], m["nsym"], m["max_nsym"])
torch.cuda.synchronize()
pay, info = pay.cpu().numpy(), info.cpu().numpy()
if mode == "dec":
    np.savez("gpurun_out/fill_ref.npz", pay=pay, info=info)
    sys.exit(0)
d = e.plan_dump(16384)
ref = np.load("gpurun_out/fill_ref.npz")
okr, ok = ref["info"][:, 4] == 1, info[:, 4] == 1
print("crc ok: old plan", okr.sum(), "packed", ok.sum(), "header", d["header"][:8])
bad = np.nonzero(okr & ~ok)[0]
print("bad", len(bad), "payload bytes equal on CRC-passing packets:",
      all((pay[p] == ref["pay"][p]).all() for p in np.nonzero(ok & okr)[0][:2000]))
