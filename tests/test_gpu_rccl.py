"""The RCCL side of the bench's multi-GPU path on the one GPU of a test box: a world-size-1
"nccl" process group (RCCL on ROCm, eager init on the rank's device as bench.py does), the
engine's decoded payloads and infos moved through the same collectives ziria_amd/node.py issues
after the timed region (all-reduce of the counts, all-gather of the row counts, padded gather
of the rows; at world size 1 node.py skips them, so they are called here directly) and
checked bit-exact.  The multi-rank logic itself is covered on gloo (tests/test_node.py); this
checks that RCCL accepts these tensors and ops on the box's GPU."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import torch.distributed as dist  # noqa: E402

from ziria_amd import node, txgen  # noqa: E402
from ziria_amd.engine import RxEngine  # noqa: E402


def test_rccl_world1_collectives_on_engine_outputs():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl" and node.comm_device(dev) == dev
        b = txgen.make_batch(300, seed=0x7CC1, device="cuda")
        e = RxEngine(0)
        e.reserve(300, b["max_nsym"])
        pay, info = e.rx(b["sym"], b["sym_off"], b["nsym"], b["max_nsym"])
        torch.cuda.synchronize()
        e.close()
        ok, bits, match = node.counts(info, 1500, pay, b["payload"])
        t = torch.tensor([ok, bits, match], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        assert t.tolist() == [300, 300 * 1500 * 8, 1]
        n = torch.tensor([pay.shape[0]], dtype=torch.int64, device=dev)
        sizes = [torch.zeros_like(n)]
        dist.all_gather(sizes, n)
        assert int(sizes[0].item()) == 300
        for rows in (pay[:, :1500].contiguous(), info):
            pad = torch.zeros((320,) + tuple(rows.shape[1:]), dtype=rows.dtype, device=dev)
            pad[:300] = rows
            blocks = [torch.empty_like(pad)]
            dist.gather(pad, blocks, dst=0)
            assert torch.equal(blocks[0][:300], rows)
        got = node.all_gather_floats([1.25, 2.5], device=dev)
        assert got == [[1.25, 2.5]]
        assert (pay[:, :1500].cpu().numpy() == b["payload"]).all() and (info[:, 4] == 1).all()
    finally:
        dist.destroy_process_group()
