"""bench.py's control flow on the CPU: main() (config 3) and bench_mixed() (config 5) with two
batches in flight, run in a subprocess with torch.cuda stubbed and the engine replaced by a
host decoder (the CPU port, identical to the oracle).  Checks the JSON line's bit-exactness
fields and the order of work: warmup steps alternating engines, then the instrumented
stage-timer pass on engine 0 alone, then exactly K timed steps alternating engines."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HARNESS = textwrap.dedent("""
    import contextlib, json, sys, types
    import torch
    sys.path.insert(0, ROOT)
    sys.argv = ["bench.py"]
    import bench
    from ziria_amd import txgen
    from oracle import oracle as O
    cpu = torch.device("cpu")
    torch.cuda.set_device = lambda *a, **k: None
    torch.cuda.synchronize = lambda *a, **k: None
    torch.cuda.Stream = lambda *a, **k: object()
    torch.cuda.stream = lambda s: contextlib.nullcontext()
    bench.torch = types.SimpleNamespace(**{k: getattr(torch, k) for k in dir(torch) if not k.startswith("__")})
    bench.torch.device = lambda *a, **k: cpu
    log = []

    class Engine:
        def __init__(self, dev):
            self.id = len([x for x in log if x[0] == "new"])
            log.append(("new", self.id))
        def reserve(self, n, s):
            pass
        def enable_timing(self, on):
            log.append(("timing", on))
        def stage_ms(self):
            return dict(signal_fft=0.01, signal_viterbi=0.03, data_fft_demap=0.13, data_viterbi=1.25,
                        descramble_crc=0.03)
        def rx(self, sym, off, nsym, S, payload, info, chan=None):
            log.append(("rx", self.id))
            pay, res = O.rx_batch_time_fast(sym.numpy(), off.numpy(), nsym.numpy(), nthreads=4)
            payload[:] = torch.from_numpy(pay)
            for i, r in enumerate(res):
                info[i, :5] = torch.tensor([r["modulation"], r["coding"], r["len"], r["err"], r["crc_ok"]])

    bench.RxEngine = Engine
    make = txgen.make_batch_range
    bench.txgen = types.SimpleNamespace(**{k: getattr(txgen, k) for k in dir(txgen) if not k.startswith("__")})
    bench.txgen.make_batch_range = lambda lo, hi, **k: make(lo, hi, **{**k, "device": cpu})
    sys.argv = ["bench.py"] + ARGS
    bench.main()
    print("LOG " + json.dumps(log))
""")


def _run(args):
    code = f"ROOT = {ROOT!r}\nARGS = {args!r}\n" + HARNESS
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = p.stdout.splitlines()
    line = json.loads(next(x for x in lines if x.startswith("{")))
    log = json.loads(next(x for x in lines if x.startswith("LOG "))[4:])
    return line, log


@pytest.mark.parametrize("args,k,w", [
    (["--npkts", "24", "--steps", "4", "--warmup", "2", "--no-cpu"], 4, 2),
    (["--config", "5", "--npkts", "40", "--steps", "3", "--warmup", "1", "--cpu-seconds", "0.2"], 3, 1),
])
def test_bench_pipelined_flow(oracle, args, k, w):
    line, log = _run(args)
    b = line["bit_exact_check"]
    assert b["payload_match"] is True and b["pipeline_outputs_equal"] is True
    assert line["steps"] == k and line["warmup"] == w and "2 batches in flight" in str(line)
    rx = [e for e in log if e[0] in ("rx", "timing")]
    on = rx.index(["timing", True])
    off = rx.index(["timing", False])
    warm, inst, timed = rx[:on], rx[on + 1:off], rx[off + 1:]
    assert [e[1] for e in warm] == [i % 2 for i in range(w)]
    assert inst and all(e == ["rx", 0] for e in inst)
    assert [e[1] for e in timed] == [(w + i) % 2 for i in range(k)]
