"""Loads libziria_rx.so (the HIP engine + C-ABI) with ctypes and declares its signatures.

There is no fallback: if the library is missing or cannot find a gfx950 device, the
calls fail loudly.  Build it with `python -m ziria_amd.build` (or __graft_entry__.build()).
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_lib", "libziria_rx.so")
# A/B timing experiments only: ZRX_LIB_VARIANT=name loads _lib/libziria_rx.<name>.so, an
# engine built from another revision by scripts/build_variant.sh.
if os.environ.get("ZRX_LIB_VARIANT"):
    LIB_PATH = os.path.join(HERE, "_lib", "libziria_rx.%s.so" % os.environ["ZRX_LIB_VARIANT"])

_lib = None

# (name, restype, argtypes) for every symbol of include/ziria_rx.h
_P = C.c_void_p
SIGNATURES = [
    ("__ext_sora_fft", None, [_P, C.c_int, _P, C.c_int]),
    ("__ext_sora_fft_dynamic", None, [_P, C.c_int, C.c_int16, _P, C.c_int]),
    ("__ext_viterbi_brick_init_fast", C.c_int, [C.c_int32, C.c_int16, C.c_int16]),
    ("__ext_viterbi_brick_decode_fast", C.c_int16, [_P, C.c_int, _P, C.c_int]),
    ("__ext_viterbiSig11a_brick_init_fast", C.c_int, [C.c_int32, C.c_int16, C.c_int16]),
    ("__ext_viterbiSig11a_brick_decode_fast", C.c_int16, [_P, C.c_int, _P, C.c_int]),
    ("__ext_v_shift_right_complex16", C.c_int, [_P, C.c_int, _P, C.c_int, C.c_int]),
    ("__ext_sora_fft64_batch", None, [_P, C.c_int, _P, C.c_int]),
    ("__ext_viterbi_batch_decode", C.c_int32,
     [_P, C.c_int, _P, C.c_int, _P, C.c_int, _P, C.c_int, _P, C.c_int, _P, C.c_int]),
    ("__ext_wifi_rx_batch", C.c_int32, [_P, C.c_int, _P, C.c_int, _P, C.c_int, _P, C.c_int]),
    ("__ext_wifi_rx_eq_batch", C.c_int32, [_P, C.c_int, _P, C.c_int, _P, C.c_int, _P, C.c_int, _P, C.c_int]),
    ("__ext_wifi_rx_stream_batch", C.c_int32, [_P, C.c_int, _P, C.c_int, C.c_int, _P, C.c_int, _P, C.c_int, _P,
                                               C.c_int]),
    ("__ext_wifi_tx_batch", C.c_int32, [_P, C.c_int, _P, C.c_int, _P, C.c_int, _P, C.c_int]),
    ("zrx_create", C.c_int, [C.POINTER(C.c_void_p), C.c_int, _P]),
    ("zrx_destroy", C.c_int, [_P]),
    ("zrx_set_stream", C.c_int, [_P, _P]),
    ("zrx_reserve", C.c_int, [_P, C.c_int, C.c_int]),
    ("zrx_enable_timing", C.c_int, [_P, C.c_int]),
    ("zrx_get_timing", C.c_int, [_P, _P]),
    ("zrx_fft64_dev", C.c_int, [_P, _P, _P, C.c_int64]),
    ("zrx_fft_dev", C.c_int, [_P, C.c_int, _P, _P, C.c_int64]),
    ("zrx_viterbi_dev", C.c_int, [_P, _P, _P, _P, C.c_int, _P, _P, _P]),
    ("zrx_plan_stats", C.c_int, [_P, _P]),
    ("zrx_plan_check", C.c_int, [_P]),
    ("zrx_pipeline_link", C.c_int, [_P, _P, C.c_int]),
    ("zrx_rx_dev", C.c_int, [_P, _P, _P, _P, C.c_int, C.c_int, _P, _P]),
    ("zrx_rx_eq_dev", C.c_int, [_P, _P, _P, _P, C.c_int, C.c_int, _P, _P, _P]),
    ("zrx_ofdm_eq_dev", C.c_int, [_P, _P, _P, _P, C.c_int, _P, _P]),
    ("zrx_rx_stream_dev", C.c_int, [_P, _P, _P, _P, C.c_int, C.c_int, C.c_int, _P, _P, _P]),
    ("zrx_cca_pattern", C.c_int, [_P]),
    ("zrx_tx_dev", C.c_int, [_P, _P, _P, C.c_int, _P, _P, _P]),
    ("zrx_tx_samples", C.c_int, [_P]),
    ("zrx_tx_preamble", C.c_int, [_P]),
    ("zrx_trig_tables", C.c_int, [_P, _P, _P]),
    ("zrx_set_devices", C.c_int, [_P, C.c_int, C.c_int64]),
    ("zrx_get_devices", C.c_int, [_P, C.c_int]),
    ("zrx_node_stats", C.c_int, [_P]),
    ("zrx_set_host_register", C.c_int, [C.c_int]),
    ("zrx_shard_split", C.c_int, [_P, C.c_int, C.c_int, C.c_int64, _P]),
    ("zrx_shard_selftest", C.c_int, [_P, C.c_int, C.c_int, C.c_int64, _P, C.c_int]),
    ("zrx_version", C.c_char_p, []),
]


class ZiriaRxError(RuntimeError):
    pass


def lib():
    """The loaded engine library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ZiriaRxError(f"{LIB_PATH} not built: run `python -m ziria_amd.build` "
                               "(the engine has no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            if os.environ.get("ZRX_LIB_VARIANT") and not hasattr(L, name):
                continue                                   # (an older revision's engine)
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        raise ZiriaRxError(f"{what} failed with code {rc}")
    return rc
