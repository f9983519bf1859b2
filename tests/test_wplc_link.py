"""The drop-in boundary as a wplc-compiled program sees it.

wplc writes `fun external` prototypes into a C++ test.cpp (src/Codegen/CgFun.hs:287-316) that
the reference builds with g++ (csrc/Makefile:92-96), so a Ziria program references the
externals by their C++-mangled names over the reference's types (num8 = char ...).
tests/wplc/wplc_caller.cpp declares them exactly that way; here it is compiled with the
reference's flags, linked against libziria_rx.so and run on the reference's KATs: the
per-call externals on the host (no GPU needed), the batched ones on the GPU."""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "wplc", "wplc_caller.cpp")

# `nm` of the reference's own objects (oracle/_ref/h_vit.o, h_fft.o: csrc/sora_ext_viterbi.cpp
# and csrc/sora_ext_lib.cpp compiled with g++ -std=c++11 as csrc/Makefile does)
REF_MANGLED = [
    "_Z14__ext_sora_fftP9complex16iS0_i",                  # sora_ext_lib.cpp:2672
    "_Z22__ext_sora_fft_dynamicP9complex16isS0_i",         # sora_ext_lib.cpp:2818
    "_Z29__ext_v_shift_right_complex16P9complex16iS0_ii",  # sora_ext_lib.cpp:1979
    "_Z29__ext_viterbi_brick_init_fastiss",                # sora_ext_viterbi.cpp:49
    "_Z31__ext_viterbi_brick_decode_fastPciPhi",           # sora_ext_viterbi.cpp:67
    "_Z35__ext_viterbiSig11a_brick_init_fastiss",          # sora_ext_viterbi.cpp:159
    "_Z37__ext_viterbiSig11a_brick_decode_fastPciPhi",     # sora_ext_viterbi.cpp:177
]


def _lib():
    import ziria_amd
    from ziria_amd import build
    build.build()
    return ziria_amd.LIB_PATH


def _defined(path):
    out = subprocess.check_output(["nm", "-D", "--defined-only", path]).decode()
    return set(re.findall(r"\bT (\S+)", out))


@pytest.fixture(scope="module")
def caller(tmp_path_factory):
    lib = _lib()
    exe = str(tmp_path_factory.mktemp("wplc") / "wplc_caller")
    libdir = os.path.dirname(lib)
    subprocess.check_call(["g++", "-std=c++11", "-Og", "-g", "-Wall", "-o", exe, SRC, "-L" + libdir, "-lziria_rx",
                           "-Wl,-rpath," + libdir])
    return exe


def test_library_exports_reference_mangled_names():
    names = _defined(_lib())
    for n in REF_MANGLED:
        assert n in names, n
    ref = [os.path.join(ROOT, "oracle", "_ref", f) for f in ("h_vit.o", "h_fft.o")]
    if all(os.path.exists(f) for f in ref):          # built from /root/reference by oracle/Makefile.ref
        out = subprocess.check_output(["nm", "--defined-only"] + ref).decode()
        want = {"__ext_sora_fft", "__ext_sora_fft_dynamic", "__ext_v_shift_right_complex16",
                "__ext_viterbi_brick_init_fast", "__ext_viterbi_brick_decode_fast",
                "__ext_viterbiSig11a_brick_init_fast", "__ext_viterbiSig11a_brick_decode_fast"}
        got = set()
        for m in re.findall(r"\bT (_Z\d+__ext_\S+)", out):
            n = re.match(r"_Z(\d+)", m)
            if m[n.end():n.end() + int(n.group(1))] in want:
                got.add(m)
        assert sorted(got) == sorted(REF_MANGLED)


def test_caller_references_resolve(caller):
    """Every __ext_ symbol the wplc-style program leaves undefined is defined by the library."""
    und = subprocess.check_output(["nm", "-u", caller]).decode()
    need = set(re.findall(r"\b(_Z\d+__ext_\w+)", und))
    assert len(need) == 9, sorted(need)
    assert need <= _defined(_lib())


def _run(caller, *args):
    r = subprocess.run([caller] + [str(a) for a in args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stderr)


def test_caller_viterbi_kat(caller, golden, tmp_path):
    k = golden["ref_kats"]
    (tmp_path / "s.bin").write_bytes(k["vit_kat_soft"].astype(np.int8).tobytes())
    _run(caller, "viterbi", tmp_path / "s.bin", 100, 0, tmp_path / "o.bin")
    bits = np.unpackbits(np.frombuffer((tmp_path / "o.bin").read_bytes(), np.uint8), bitorder="little")
    assert (bits == k["vit_kat_bits"]).all()


def test_caller_viterbi_reference_frames(caller, golden, tmp_path):
    g = golden["ref_viterbi"]
    cases, so, oo = g["vit_cases"], g["vit_soft_off"], g["vit_out_off"]
    for i, (cr, fl, noise) in enumerate(cases):
        if fl not in (3, 1500) or noise not in (0, 7):
            continue
        (tmp_path / "s.bin").write_bytes(g["vit_soft"][so[i]:so[i + 1]].astype(np.int8).tobytes())
        _run(caller, "viterbi", tmp_path / "s.bin", int(fl), int(cr), tmp_path / "o.bin")
        got = np.frombuffer((tmp_path / "o.bin").read_bytes(), np.uint8)
        exp = g["vit_out"][oo[i]:oo[i + 1]]
        assert (got[:exp.size] == exp).all(), (cr, fl, noise)


def test_caller_signal_kat(caller, golden, tmp_path):
    k = golden["ref_kats"]
    (tmp_path / "s.bin").write_bytes(k["sig_kat_soft"].astype(np.int8).tobytes())
    _run(caller, "sig", tmp_path / "s.bin", tmp_path / "o.bin")
    bits = np.unpackbits(np.frombuffer((tmp_path / "o.bin").read_bytes(), np.uint8), bitorder="little")[:24].copy()
    bits[18:] = 0
    assert (bits == k["sig_kat_bits"]).all()


def test_caller_fft_kat_all_sizes(caller, golden, tmp_path):
    g = golden["ref_fftn"]
    off = 0
    for n in g["sizes"]:
        n = int(n)
        (tmp_path / "x.bin").write_bytes(np.ascontiguousarray(g["kat_in"][off:off + n], np.int16).tobytes())
        _run(caller, "fft", tmp_path / "x.bin", n, tmp_path / "y.bin")
        got = np.frombuffer((tmp_path / "y.bin").read_bytes(), np.int16).reshape(-1, 2)
        assert (got == g["kat_out"][off:off + n]).all(), n
        off += n


def test_caller_shift_right(caller, oracle, tmp_path):
    x = np.random.default_rng(8).integers(-32768, 32768, (13, 2)).astype(np.int16)
    (tmp_path / "x.bin").write_bytes(x.tobytes())
    for sh in (0, 3, 15):
        _run(caller, "shift", tmp_path / "x.bin", sh, tmp_path / "z.bin")
        got = np.frombuffer((tmp_path / "z.bin").read_bytes(), np.int16).reshape(-1, 2)
        assert (got == oracle.v_shift_right_complex16(x, sh)).all(), sh


@pytest.mark.gpu
def test_caller_batched_viterbi_kat(caller, golden, tmp_path):
    """The batched external, C++ linkage, on the GPU: the Viterbi KAT as a one-packet batch."""
    k = golden["ref_kats"]
    (tmp_path / "s.bin").write_bytes(k["vit_kat_soft"].astype(np.int8).tobytes())
    _run(caller, "vbatch", tmp_path / "s.bin", 100, 0, tmp_path / "o.bin")
    bits = np.unpackbits(np.frombuffer((tmp_path / "o.bin").read_bytes(), np.uint8), bitorder="little")
    kat = k["vit_kat_bits"]                         # the KAT's ground file holds the first 256 bits
    assert bits.size == 800 and (bits[:kat.size] == kat).all()


@pytest.mark.gpu
def test_caller_batched_rx_chain_fixture(caller, golden, tmp_path):
    """__ext_wifi_rx_batch (C++ linkage) on the reference-brick chain fixture."""
    g = golden["ref_chain"]
    sym, off, nsym = g["mix_sym"], g["mix_off"], g["mix_nsym"]
    (tmp_path / "sym.bin").write_bytes(np.ascontiguousarray(sym, np.int16).tobytes())
    csr = np.concatenate([off, [off[-1] + nsym[-1]]]).astype(np.int64)
    (tmp_path / "m.txt").write_text(" ".join(str(int(v)) for v in csr))
    _run(caller, "rx", tmp_path / "sym.bin", tmp_path / "m.txt", tmp_path / "p.bin", tmp_path / "i.bin")
    pay = np.frombuffer((tmp_path / "p.bin").read_bytes(), np.uint8).reshape(-1, 4096)
    info = np.frombuffer((tmp_path / "i.bin").read_bytes(), np.int32).reshape(-1, 8)
    assert (info[:, 4] == g["mix_crc"]).all()
    po = g["mix_payload_off"]
    for i in range(len(off)):
        e = g["mix_payload"][po[i]:po[i + 1]]
        assert (pay[i, :e.size] == e).all(), i


@pytest.mark.gpu
def test_caller_static_arrays_registered(caller, tmp_path):
    """A wplc program keeps its arrays in static storage; __ext_wifi_rx_batch page-locks that
    storage once (zrx_set_host_register mode 1, the default) and copies straight from and to
    it on every later call, and a rewrite of the arrays between calls is seen by the next one.
    2048 config-3 packets (30 MB of symbols) in the caller's .bss, three calls."""
    import torch
    from ziria_amd import txgen
    b = txgen.make_batch(2048, seed=0x51A7, sigma=4.0, device="cuda")
    S = b["max_nsym"]
    (tmp_path / "sym.bin").write_bytes(np.ascontiguousarray(b["sym"].cpu().numpy()).tobytes())
    (tmp_path / "m.txt").write_text(" ".join(str(i * S) for i in range(2049)))
    del b["sym"]
    torch.cuda.empty_cache()
    _run(caller, "rxstatic", tmp_path / "sym.bin", tmp_path / "m.txt", tmp_path / "p.bin", tmp_path / "i.bin",
         tmp_path / "log.txt")
    calls = [ln.split() for ln in (tmp_path / "log.txt").read_text().splitlines()]
    rc = [int(c[3]) for c in calls]
    st = [[int(x) for x in c[7:15]] for c in calls]          # zrx_node_stats after each call
    assert rc == [2048, 2048, 2047]
    # mode 1; the static segment registered once (one range, >= the 38 MB of arrays), then hits
    # stats: {shards, mode, ranges held, bytes held, registrations, hits, failures, min_shard_bytes}
    assert st[0][1] == 1 and st[0][2] == 1 and st[0][3] >= 2048 * 57 * 256 + 2048 * 4096
    assert st[0][4] == st[2][4] and st[2][2] == 1 and st[2][6] == 0
    assert st[1][5] - st[0][5] == 3 and st[2][5] - st[1][5] == 3      # sym, payload, info: in place
    pay = np.frombuffer((tmp_path / "p.bin").read_bytes(), np.uint8).reshape(-1, 4096)
    assert (pay[:, :1500] == b["payload"]).all()
    info = np.frombuffer((tmp_path / "i.bin").read_bytes(), np.int32).reshape(-1, 8)
    assert info[5, 4] == 0 and (np.delete(info[:, 4], 5) == 1).all()
