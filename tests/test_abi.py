"""The C-ABI library loads and exports every symbol include/ziria_rx.h declares (no
compute calls: this runs without a GPU)."""
import ctypes
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(ROOT, "include", "ziria_rx.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b((?:__ext_|zrx_)\w+)\s*\(", txt)))


def test_library_exports_declared_symbols():
    import ziria_amd
    from ziria_amd import build
    build.build()
    lib = ctypes.CDLL(ziria_amd.LIB_PATH)
    names = _declared()
    assert len(names) >= 18
    for n in names:
        assert hasattr(lib, n), n
    out = subprocess.check_output(["nm", "-D", "--defined-only", ziria_amd.LIB_PATH]).decode()
    for n in names:
        assert re.search(rf"\bT {n}\b", out), n


def test_python_signatures_cover_header():
    from ziria_amd._lib import SIGNATURES
    assert sorted(n for n, _, _ in SIGNATURES) == _declared()


def test_no_gpu_fails_loudly():
    """On a machine without a gfx950 device the engine refuses instead of computing on the CPU."""
    import torch
    if torch.cuda.is_available():
        return
    import ziria_amd
    h = ctypes.c_void_p()
    assert ziria_amd.lib().zrx_create(ctypes.byref(h), 0, None) == -4      # ZRX_ENODEV
