"""The batching hook inside the reference's own driver (north_star: "a batching hook in
driver.cpp").  oracle/Makefile.hook compiles the reference runtime
(csrc/driver.cpp with integration/csrc/driver.cpp.patch applied, params.c, buf_*.c, ...)
from /root/reference with integration/csrc/hip_ext_batch.cpp and a stub wplc program, linked
against libziria_rx.so.  Without --batch-mode the patched main runs the reference's stream
path unchanged; with it, one batched GPU call decodes the input file."""
import os
import subprocess

import numpy as np
import pytest

from tests.test_driver import _vals


@pytest.fixture(scope="module")
def hooked():
    from oracle import oracle as O
    from ziria_amd import build
    build.build()
    exe = O.build_hook()
    if exe is None:
        pytest.skip("reference driver not built (needs /root/reference in the build container)")
    return exe


def _run(exe, args, rc=0):
    r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=120)
    assert r.returncode == rc, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    return r


def test_stream_path_unchanged(hooked):
    """No --batch-mode: the reference's main parses its flags and runs wpl_go() (driver.cpp:282)."""
    r = _run(hooked, ["--input=dummy", "--output=dummy", "--dummy-samples=10"])
    assert "Bytes copied:" in r.stdout and "Time elapsed (usec)" in r.stdout


def test_batch_mode_file_formats(hooked, tmp_path):
    src = tmp_path / "in.dbg"
    src.write_text("1, -2,3\n-32768,32767,\n0,5")
    out = tmp_path / "out.dbg"
    _run(hooked, ["--batch-mode=dry-run", f"--input-file-name={src}", "--input-file-mode=dbg",
                  f"--output-file-name={out}", "--output-file-mode=dbg", "--heap-size=1000000"])
    assert out.read_text() == "1,-2,3,-32768,32767,0,5"
    _run(hooked, ["--batch-mode=packets", "--bogus-flag"], rc=2)


def test_batch_mode_without_gpu_fails_cleanly(hooked, tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("has a GPU")
    src = tmp_path / "sym.bin"
    np.zeros(128 * 5, np.int16).tofile(src)
    r = _run(hooked, ["--batch-mode=packets", f"--input-file-name={src}", f"--output-file-name={tmp_path / 'o'}"], rc=1)
    assert "engine error -4" in r.stderr


@pytest.mark.gpu
def test_batch_mode_receiver_kats(hooked, tmp_path, golden):
    """code/WiFi/tests/test_rx and test_real_rx through the reference driver's batching hook:
    the reference's .infile in, its ground output out."""
    fe = golden["ref_fe"]
    cases = (("rx", ["--batch-idle=1000", "--batch-downsample"]),
             ("real", ["--batch-idle=1000", "--batch-scale=10", "--batch-max-bytes=10"]))
    for tag, extra in cases:
        src = tmp_path / f"{tag}.infile"
        src.write_text(",".join(str(v) for v in fe[f"{tag}_in"].reshape(-1)))
        out = tmp_path / f"{tag}.outfile"
        _run(hooked, ["--batch-mode=receiver", f"--input-file-name={src}", "--input-file-mode=dbg",
                      f"--output-file-name={out}", "--output-file-mode=dbg"] + extra)
        got = _vals(out.read_text()).astype(np.int8).view(np.uint8)
        assert (got == fe[f"{tag}_out"]).all(), tag


def test_program_binds_library_fft(hooked, tmp_path, golden):
    """The FFT half of the drop-in: the stub program is compiled as wplc output is (through
    csrc/common.h, which #includes sora_ext_lib.cpp), with integration/csrc/sora_ext_lib.cpp.patch
    and -DZIRIA_HIP_EXT, so __ext_sora_fft and __ext_sora_fft_dynamic are undefined in the
    executable and bind to libziria_rx.so; run through the reference driver's stream path, the
    program's FFT of the tests/libs/test_fft KAT and of the 42-size KAT equals the ground."""
    nm = subprocess.check_output(["nm", hooked]).decode()
    for sym in ("_Z14__ext_sora_fftP9complex16iS0_i", "_Z22__ext_sora_fft_dynamicP9complex16isS0_i"):
        assert any(ln.split()[-2:] == ["U", sym] for ln in nm.splitlines()), sym
    kat = golden["ref_kats"]
    fn = golden["ref_fftn"]
    cases = [(64, kat["fft64_kat_in"], kat["fft64_kat_out"])]
    off = 0
    for n in fn["sizes"]:
        cases.append((int(n), fn["kat_in"][off:off + n], fn["kat_out"][off:off + n]))
        off += int(n)
    assert off == fn["kat_in"].shape[0]
    for n, x, y in cases:
        src, dst = tmp_path / f"in{n}.bin", tmp_path / f"out{n}.bin"
        np.asarray(x, "<i2").tofile(src)
        env = dict(os.environ, ZRX_STUB_FFT_IN=str(src), ZRX_STUB_FFT_OUT=str(dst), ZRX_STUB_FFT_N=str(n))
        r = subprocess.run([hooked, "--input=dummy", "--output=dummy", "--dummy-samples=10"], env=env,
                           capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, (n, r.returncode, r.stderr[-500:])
        assert (np.fromfile(dst, "<i2").reshape(-1, 2) == y).all(), n
