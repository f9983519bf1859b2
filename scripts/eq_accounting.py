"""Accounts for the round-4 `bench.py --eq` bit-exact flag: decodes the
bench's two EQ batches (the exact packets bench.py builds on the GPU) with the CPU port and
counts, per batch, the CRC failures and the failures whose payload bytes still equal what was
sent (errors only in the CRC field), then what the round-4 check computed when batch 0's
payloads were judged against batch 1's CRC flags.  One GPU run; prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ziria_amd import txgen  # noqa: E402
from oracle import oracle as O  # noqa: E402

res = {}
for seed in (0x5EED, 0x5EEE):
    b = txgen.make_batch_range(0, 16384, mod=3, coding=2, payload_len=1500, sigma=2.0, seed=seed, device="cuda",
                               channel=True)
    pay, r = O.rx_batch_time_eq_fast(b["sym"].cpu().numpy(), b["sym_off"].cpu().numpy(), b["nsym"].cpu().numpy(),
                                     b["chan"].cpu().numpy(), nthreads=16)
    crc = np.array([x["crc_ok"] for x in r], bool)
    same = (pay[:, :1500] == b["payload"]).all(1)
    res[seed] = (crc, same)
(c0, s0), (c1, s1) = res[0x5EED], res[0x5EEE]
print(json.dumps({"batch0_crc_fail": int((~c0).sum()), "batch0_fail_payload_equal": int((~c0 & s0).sum()),
                  "batch1_crc_fail": int((~c1).sum()), "batch1_fail_payload_equal": int((~c1 & s1).sum()),
                  "crc_pass_both": int(c0.sum() + c1.sum()),
                  "round4_aliased_check_flagged": int((c1 & ~s0).sum()),
                  "crc_passing_payload_mismatch": int((c0 & ~s0).sum() + (c1 & ~s1).sum())}))
