"""bench.py's control flow on the CPU: main() (configs 3 and 4) and bench_mixed() (config 5)
with two batches in flight, run in a subprocess with torch.cuda stubbed and the engine
replaced by a host decoder (the CPU port, identical to the oracle).  Checks the JSON line's
bit-exactness fields and the order of work: the streams ordered after the inputs, warmup
steps alternating engines and input batches, the instrumented stage-timer pass on engine 0
alone, exactly K timed steps, the per-batch verification passes and the single-engine pass;
and `bench.py --gpus 2` starting two ranks itself (gloo in place of RCCL)."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HARNESS = textwrap.dedent("""
    import contextlib, json, os, sys, types
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    argv = sys.argv[1:]
    sys.argv = ["bench.py"]
    import bench
    from ziria_amd import txgen
    from oracle import oracle as O
    cpu = torch.device("cpu")
    log = []

    class Stream:
        def __init__(self, *a, **k):
            self.id = len([x for x in log if x[0] == "stream"])
            log.append(("stream", self.id))
        def wait_stream(self, other):
            log.append(("wait_stream", self.id))

    torch.cuda.set_device = lambda *a, **k: None
    torch.cuda.synchronize = lambda *a, **k: None
    torch.cuda.Stream = Stream
    torch.cuda.current_stream = lambda *a, **k: "current"
    torch.cuda.stream = lambda s: contextlib.nullcontext()
    torch.cuda.empty_cache = lambda *a, **k: None

    class Event:                                  # (host clock in place of a HIP event)
        def __init__(self, **k):
            self.t = 0.0
        def record(self, stream=None):
            import time
            self.t = time.perf_counter()
        def elapsed_time(self, other):
            return (other.t - self.t) * 1e3

    torch.cuda.Event = Event
    torch.cuda.get_device_properties = lambda d: types.SimpleNamespace(pci_domain_id=0, pci_bus_id=0x11 + int(
        os.environ.get("RANK", "0")), pci_device_id=0, name="stub")
    bench.torch = types.SimpleNamespace(**{k: getattr(torch, k) for k in dir(torch) if not k.startswith("__")})
    bench.torch.device = lambda *a, **k: cpu
    init = dist.init_process_group
    bench.dist = types.SimpleNamespace(**{k: getattr(dist, k) for k in dir(dist) if not k.startswith("__")})
    bench.dist.init_process_group = lambda *a, **k: init("gloo")
    batches = {}

    class Engine:
        def __init__(self, dev):
            self.id = len([x for x in log if x[0] == "new"])
            log.append(("new", self.id))
        def reserve(self, n, s):
            pass
        def close(self):
            log.append(("close", self.id))
        def link(self, other, mode):
            log.append(("link", self.id, other.id, mode))
        def plan_check(self):
            log.append(("plan_check", self.id))
        def enable_timing(self, on):
            log.append(("timing", on))
        def stage_ms(self):
            return dict(signal_fft=0.01, signal_viterbi=0.03, data_fft_demap=0.13, data_viterbi=1.25,
                        descramble_crc=0.03)
        def rx(self, sym, off, nsym, S, payload, info, chan=None):
            b = batches.setdefault(sym.data_ptr(), len(batches))
            log.append(("rx", self.id, b))
            pay, res = O.rx_batch_time_fast(sym.numpy(), off.numpy(), nsym.numpy(), nthreads=4)
            payload[:] = torch.from_numpy(pay)
            for i, r in enumerate(res):
                info[i, :5] = torch.tensor([r["modulation"], r["coding"], r["len"], r["err"], r["crc_ok"]])

        def viterbi(self, soft, soft_off, params, out, out_off, out_bits):
            b = batches.setdefault(soft.data_ptr(), len(batches))
            log.append(("vit", self.id, b))
            n = soft_off.numel()
            p = params.numpy()
            o = O.viterbi_batch(soft.numpy(), soft_off.numpy(), p[:, 2], p[:, 0], p[:, 1], out_off.numpy(),
                                out.numel(), nthreads=4, fast=True)
            out[:] = torch.from_numpy(o)
            out_bits[:] = torch.from_numpy(p[:, 0] * 8)

    bench.RxEngine = Engine
    make, mixed = txgen.make_batch_range, txgen.make_mixed_fast
    bench.txgen = types.SimpleNamespace(**{k: getattr(txgen, k) for k in dir(txgen) if not k.startswith("__")})
    bench.txgen.make_batch_range = lambda lo, hi, **k: make(lo, hi, **{**k, "device": cpu})
    bench.txgen.make_mixed_fast = lambda n, **k: mixed(n, **{**k, "device": cpu})
    sys.argv = [os.path.abspath(__file__)] + argv
    bench.main()
    # (each rank's log to a file of its own: ranks share the stdout pipe, and a long line of
    # one rank can land inside another's)
    with open(os.path.join(os.environ["ZRX_FLOW_LOGDIR"], "log_%s.json" % os.environ.get("RANK", "0")), "w") as f:
        f.write(json.dumps(log))
""")


def _run(tmp_path, args):
    script = tmp_path / "bench_harness.py"
    script.write_text(f"ROOT = {ROOT!r}\n" + HARNESS)
    env = dict(os.environ, OMP_NUM_THREADS="2", ZRX_FLOW_LOGDIR=str(tmp_path))
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, str(script)] + args, capture_output=True, text=True, timeout=900, cwd=ROOT,
                       env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = p.stdout.splitlines()
    line = json.loads(next(x for x in lines if x.startswith("{")))
    logs = {}
    for f in tmp_path.glob("log_*.json"):
        logs[int(f.stem[4:])] = json.loads(f.read_text())
    return line, logs


@pytest.mark.parametrize("args,k,w", [
    (["--npkts", "24", "--steps", "4", "--warmup", "2", "--no-cpu", "--no-sub"], 4, 2),
    (["--config", "5", "--npkts", "40", "--steps", "3", "--warmup", "1", "--cpu-seconds", "0.2", "--pipeline", "2"], 3, 1),
])
def test_bench_pipelined_flow(oracle, tmp_path, args, k, w):
    line, logs = _run(tmp_path, args)
    log = logs[0]
    b = line["bit_exact_check"]
    assert b["payload_match"] is True and b["pipeline_outputs_equal"] is True
    assert line["steps"] == k and line["warmup"] == w and "2 batches in flight" in str(line)
    nb = 2
    # both engine streams wait for the current stream before the first launch
    first_rx = next(i for i, e in enumerate(log) if e[0] == "rx")
    assert sorted(e[1] for e in log[:first_rx] if e[0] == "wait_stream") == [0, 1]
    rx = [e for e in log if e[0] in ("rx", "timing")]
    on = rx.index(["timing", True])
    off = rx.index(["timing", False])
    warm, inst, rest = rx[:on], rx[on + 1:off], rx[off + 1:]
    settle = warm[w:]                               # untimed launches on engine 0 before the timers (clock ramp)
    warm = warm[:w]
    assert [e[1:] for e in warm] == [[i % 2, i % nb] for i in range(w)]
    assert len(inst) >= 3 * nb and all(e[1] == 0 for e in inst) and sorted({e[2] for e in inst}) == [0, 1]
    assert [e[1:] for e in settle] == [[0, i % nb] for i in range(len(inst))]
    timed = rest[:k]
    assert [e[1:] for e in timed] == [[(w + i) % 2, (w + i) % nb] for i in range(k)]
    if "--config" in args:                          # config 5: engine 0 alone over the timed batches, then the checks
        assert ["link", 0, 1, 4] in log
        assert [e[1:] for e in rest[k:2 * k]] == [[0, (w + i) % nb] for i in range(k)]
        assert line["value_one_engine"] > 0
        rest = rest[k:]
    verify = rest[k:k + 2 * nb]
    assert [e[1:] for e in verify] == [[j, bi] for bi in range(nb) for j in range(2)]
    if "--config" not in args:                      # config 3: the single-engine pass, K steps on engine 0
        assert ["link", 0, 1, 9] in log and ["plan_check", 0] in log and ["plan_check", 1] in log
        single = rest[k + 2 * nb:]                  # its own warmup, then the K timed steps
        assert [e[1:] for e in single] == [[0, i % nb] for i in range(w)] + [[0, i % nb] for i in range(k)]
        assert line["config"]["batches_per_gpu"] == nb and b["packets"] == nb * 24
        assert line["value_one_engine"] > 0


def test_bench_viterbi_only_flow(oracle, tmp_path):
    """Config 2: two soft batches, two engines; the steps alternate engines and batches and
    every frame of both batches is checked on both engines."""
    line, logs = _run(tmp_path, ["--config", "2", "--npkts", "8", "--payload", "100", "--steps", "3",
                                 "--warmup", "1", "--cpu-seconds", "0.2"])
    log = [e[1:] for e in logs[0] if e[0] == "vit"]
    assert log[:4] == [[i % 2, i % 2] for i in range(4)]
    assert log[4:] == [[j, b] for b in range(2) for j in range(2)]
    assert line["bit_exact_check"]["frames_equal_sent"] is True and line["config"]["batches"] == 2
    assert line["cpu_baseline"]["value"] > 0


def test_bench_gpus2_spawns_two_ranks(oracle, tmp_path):
    """`bench.py --gpus 2` with no launcher starts two ranks itself (torch.distributed.run as a
    child); rank 0 gathers every packet of both ranks' shards and prints one line for 2 GPUs
    (the CPU baseline belongs to the N = 1 line only)."""
    line, logs = _run(tmp_path, ["--gpus", "2", "--npkts", "12", "--steps", "2", "--warmup", "1",
                                 "--cpu-seconds", "0.2"])
    assert sorted(logs) == [0, 1]
    assert line["n_gpus"] == 2 and line["config"]["packets_total"] == 24 and line["config"]["packets_per_gpu"] == 12
    b = line["bit_exact_check"]
    assert b["packets"] == 2 * 24 and b["crc_pass"] == 2 * 24 and b["payload_match"] is True
    assert b["mismatched_packets"] == 0
    assert line["cpu_baseline"] is None and "N = 1" in line["cpu_baseline_note"]
    # every rank's device and PCI address, and its own time over the timed region
    assert [d["rank"] for d in line["devices"]] == [0, 1]
    assert [d["pci"] for d in line["devices"]] == ["0000:11:00.0", "0000:12:00.0"]
    assert all(d["elapsed_s"] > 0 for d in line["devices"])
    assert "sub_results" not in line
    for r in (0, 1):
        assert any(e[0] == "rx" for e in logs[r])
    # the same run also decodes config 4 as SURVEY §8(d) defines it: npkts packets in all,
    # split over the ranks, every gathered packet checked
    st = line["strong"]
    assert st["scaling"] == "strong" and st["config"]["packets_total"] == 12 and st["config"]["packets_per_gpu"] == 6
    assert st["bit_exact_check"]["packets"] == 2 * 12 and st["bit_exact_check"]["payload_match"] is True
    assert st["value"] > 0 and st["ms_per_step"] > 0


def test_bench_share_gpu_two_ranks(oracle, tmp_path):
    """--share-gpu: both ranks on GPU 0 over a gloo group (the multi-rank path on a one-GPU
    box): labelled as one GPU and no scaling point, every gathered packet checked."""
    line, logs = _run(tmp_path, ["--gpus", "2", "--share-gpu", "--npkts", "10", "--steps", "2", "--warmup", "1",
                                 "--no-cpu"])
    assert sorted(logs) == [0, 1]
    assert line["n_gpus"] == 1 and line["ranks"] == 2 and "no scaling point" in line["multi_rank_mode"]
    assert line["bit_exact_check"]["packets"] == 2 * 20 and line["bit_exact_check"]["payload_match"] is True
    assert line["strong"]["bit_exact_check"]["packets"] == 2 * 10


def test_bench_one_engine_flow(oracle, tmp_path):
    """--pipeline 1 (auto's choice at 8192 packets per GPU and above): one engine, no link,
    the timed steps and the verification all on engine 0."""
    line, logs = _run(tmp_path, ["--npkts", "24", "--steps", "3", "--warmup", "1", "--no-cpu", "--pipeline", "1",
                                 "--no-sub"])
    log = logs[0]
    assert "1 batch in flight" in line["config"]["pipeline"]
    assert not any(e[0] == "link" for e in log) and all(e[1] == 0 for e in log if e[0] == "rx")
    assert line["bit_exact_check"]["payload_match"] is True and line["value_one_engine"] > 0


def test_bench_default_line_carries_sub_results(oracle, tmp_path):
    """The default one-GPU line: the headline plus configs 2 and 5 and the two config-4 shard
    sizes as sub-results, each with its own bit-exact check, ms_per_step and per-step times
    (npkts 32 here: shards of 4 and 8 packets)."""
    line, logs = _run(tmp_path, ["--npkts", "32", "--payload", "200", "--steps", "2", "--warmup", "1", "--no-cpu"])
    st = line["step_stats"]["gpu_step_ms"]
    assert st["min"] <= st["median"] <= st["max"] and line["step_stats"]["host_issue_ms"]["max"] >= 0
    assert line["devices"][0]["pci"] == "0000:11:00.0"
    sub = line["sub_results"]
    assert sorted(k for k in sub if k != "wall_s") == ["config2", "config5", "shard_4", "shard_8"]
    assert sub["config2"]["bit_exact_check"]["frames_equal_sent"] is True
    assert sub["config5"]["bit_exact_check"]["payload_match"] is True
    assert sub["config5"]["bit_exact_check"]["oracle_sample_match"] is True
    for k in ("shard_4", "shard_8"):
        b = sub[k]["bit_exact_check"]
        assert b["payload_match"] is True and b["mismatched_packets"] == 0 and b["packets"] == 2 * int(k[6:])
    for k in ("config2", "config5", "shard_4", "shard_8"):
        assert "error" not in sub[k] and sub[k]["command"].startswith("bench.py ")     # (its own child process)
        assert sub[k]["ms_per_step"] > 0 and sub[k]["value"] > 0
        g = sub[k]["step_stats"]["gpu_step_ms"]
        assert g["min"] <= g["median"] <= g["max"]
