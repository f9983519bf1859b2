"""The batching driver: the driver.cpp hook of
integration/csrc/hip_ext_batch.cpp as the standalone program tools/ziria_rx_driver.cpp; the
reference's dbg and bin file formats (csrc/buf_numerics16.c, buf_numerics8.c) and packet
manifests in front of the engine.  The format round trips run on the CPU; the KAT runs need
the GPU.  tests/test_driver_hook.py runs the same hook inside the reference's own driver."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _driver():
    if os.environ.get("ZRX_DRIVER"):                   # e.g. the sanitizer build (make asan)
        return os.environ["ZRX_DRIVER"]
    from ziria_amd import build
    build.build()
    return build.DRIVER


def _run(args):
    r = subprocess.run([_driver()] + args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return r


def _vals(text):
    return np.array([int(v) for v in text.replace("\n", ",").split(",") if v.strip()], np.int64)


def test_dbg_round_trip(tmp_path):
    src = tmp_path / "in.dbg"
    src.write_text("1, -2,3\n-32768,32767,\n0,5")        # spaces, newlines, trailing comma
    out = tmp_path / "out.dbg"
    _run([f"--input-file-name={src}", "--input-file-mode=dbg", f"--output-file-name={out}",
          "--output-file-mode=dbg", "--batch-mode=dry-run"])
    assert out.read_text() == "1,-2,3,-32768,32767,0,5"


def test_bin_round_trip(tmp_path):
    x = np.random.default_rng(1).integers(-32768, 32768, 1000).astype(np.int16)
    src = tmp_path / "in.bin"
    x.tofile(src)
    out = tmp_path / "out.bin"
    _run([f"--input-file-name={src}", "--input-file-mode=bin", f"--output-file-name={out}",
          "--output-file-mode=bin", "--batch-mode=dry-run"])
    assert (np.fromfile(out, np.int16) == x).all()


def test_bad_arguments_fail():
    for args in (["--nonsense"], ["--batch-mode=packets", "--nonsense"], ["--batch-mode=bogus"]):
        r = subprocess.run([_driver()] + args, capture_output=True, text=True, timeout=60)
        assert r.returncode == 2, args


@pytest.mark.gpu
def test_driver_receiver_kats(tmp_path, golden):
    """test_rx: read >>> append_idle >>> downSample >>> receiver >>> convert_to_int8 >>> write;
    test_real_rx: append_idle (x10) >>> receiver >>> print_hdr (10 bytes).  The driver turns
    the reference's own .infile into its ground output."""
    fe = golden["ref_fe"]
    cases = (("rx", ["--batch-idle=1000", "--batch-downsample"]),
             ("real", ["--batch-idle=1000", "--batch-scale=10", "--batch-max-bytes=10"]))
    for tag, extra in cases:
        src = tmp_path / f"{tag}.infile"
        src.write_text(",".join(str(v) for v in fe[f"{tag}_in"].reshape(-1)))
        out = tmp_path / f"{tag}.outfile"
        _run([f"--input-file-name={src}", "--input-file-mode=dbg", f"--output-file-name={out}",
              "--output-file-mode=dbg", "--batch-mode=receiver"] + extra)
        got = _vals(out.read_text()).astype(np.int8).view(np.uint8)
        assert (got == fe[f"{tag}_out"]).all(), tag


@pytest.mark.gpu
def test_driver_packets_manifest(tmp_path, golden):
    """Packet mode over a manifest of CP-removed symbol ranges (the chain fixture)."""
    g = golden["ref_chain"]
    sym, off, nsym = g["mix_sym"], g["mix_off"], g["mix_nsym"]
    src = tmp_path / "sym.bin"
    sym.astype(np.int16).tofile(src)
    man = tmp_path / "pkts.txt"
    man.write_text("".join(f"{o} {n}\n" for o, n in zip(off, nsym)))
    out, inf = tmp_path / "pay.bin", tmp_path / "info.txt"
    _run([f"--input-file-name={src}", "--input-file-mode=bin", f"--output-file-name={out}",
          "--output-file-mode=bin", "--batch-mode=packets", f"--batch-manifest={man}",
          f"--batch-info-file={inf}"])
    info = np.array([[int(v) for v in l.split(",")] for l in inf.read_text().split()], np.int64)
    assert (info[:, 4] == g["mix_crc"]).all()
    got = np.fromfile(out, np.uint8)
    exp = np.concatenate([g["mix_payload"][g["mix_payload_off"][i]:g["mix_payload_off"][i + 1]]
                          for i in range(len(off)) if info[i, 3] == 0 and info[i, 5] == 0])
    assert got.size == exp.size and (got == exp).all()
