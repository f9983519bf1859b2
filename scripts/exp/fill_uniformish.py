"""Probe: the packed plan's per-column cost.  A config-3 batch with one packet replaced by a
shorter frame is a mixed batch, so it takes the mixed plans, but its waves are whole groups of
equal frames (no seams): with ZRX_FILL=1 (packed rows) and ZRX_FILL=0 (rows of frames) the
Viterbi does the same work as the uniform batch.  Prints the data-Viterbi stage time of each
(children, so each gets its own context) and of the uniform batch."""
import json
import os
import subprocess
import sys

sys.path.insert(0, ".")
if len(sys.argv) == 1:
    for f in ("1", "0", "u"):
        r = subprocess.run([sys.executable, __file__, f], env=dict(os.environ, ZRX_FILL=f if f != "u" else "1"))
        assert r.returncode == 0
    sys.exit(0)
import torch  # noqa: E402
from ziria_amd import txgen  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402

dev = torch.device("cuda", 0)
b = txgen.make_batch_range(0, 16384, payload_len=1500, seed=0x5EED, device=dev)
sym, off, nsym, S = b["sym"], b["sym_off"].clone(), b["nsym"].clone(), b["max_nsym"]
if sys.argv[1] != "u":
    o = txgen.make_batch_range(0, 1, payload_len=1000, seed=0x77, device=dev)
    off[0] = sym.shape[0]
    nsym[0] = o["nsym"][0]
    sym = torch.cat([sym, o["sym"][: int(o["nsym"][0])]], 0)
e = RxEngine(0)
e.reserve(16384, S)
for _ in range(20):
    pay, info = e.rx(sym, off, nsym, S)
torch.cuda.synchronize()
e.enable_timing(True)
for _ in range(10):
    pay, info = e.rx(sym, off, nsym, S)
torch.cuda.synchronize()
st = e.stage_ms()
ok = int((info[:, 4] == 1).sum().item())
print(json.dumps({"fill": sys.argv[1], "data_viterbi": round(st["data_viterbi"], 4), "crc_ok": ok,
                  "plan": e.plan_stats()}), flush=True)
