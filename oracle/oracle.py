"""ORACLE — test infrastructure only.

ctypes wrapper around oracle/_build/libziria_oracle.so (the scalar C restatement of the
reference hot path, oracle/ziria_oracle.c) and, when present, oracle/_ref/libzref.so (the
reference bricks compiled from /root/reference/csrc by oracle/Makefile.ref).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product package (ziria_amd) never does.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "_build", "libziria_oracle.so")
_REF = os.path.join(_HERE, "_ref", "libzref.so")
_lib = None
_ref = None


def build(quiet=True):
    """Compile the C restatement (and the reference bricks when /root/reference exists)."""
    out = subprocess.DEVNULL if quiet else None
    subprocess.check_call(["make", "-C", _HERE], stdout=out)
    if os.path.isdir("/root/reference/csrc"):
        subprocess.check_call(["make", "-C", _HERE, "-f", "Makefile.ref"], stdout=out, stderr=out)


HOOKED_DRIVER = os.path.join(_HERE, "_ref", "driver_hooked")


def build_hook(quiet=True):
    """The reference's own driver (csrc/driver.cpp + runtime, from /root/reference) with the
    batching hook of integration/csrc linked against libziria_rx.so (oracle/Makefile.hook).
    Returns the binary's path, or None where /root/reference is absent and it was not built
    before (a GPU box runs the binary built here)."""
    if os.path.isdir("/root/reference/csrc"):
        out = subprocess.DEVNULL if quiet else None
        subprocess.check_call(["make", "-C", _HERE, "-f", "Makefile.hook"], stdout=out)
    return HOOKED_DRIVER if os.path.exists(HOOKED_DRIVER) else None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        _lib = C.CDLL(_LIB)
        _lib.zo_crc32_bits.restype = C.c_uint32
        _lib.zo_lut.restype = C.POINTER(C.c_uint8)
    return _lib


def ref():
    """The compiled reference bricks, or None if they were not built here."""
    global _ref
    if _ref is None and os.path.exists(_REF):
        _ref = C.CDLL(_REF)
    return _ref


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class RxResult(C.Structure):
    _fields_ = [("coding", C.c_int32), ("modulation", C.c_int32), ("len", C.c_int32),
                ("err", C.c_int32), ("crc_ok", C.c_int32), ("nsym_used", C.c_int32),
                ("viterbi_bits", C.c_int32)]


class Vit(C.Structure):
    _fields_ = [("m", C.c_uint8 * 64), ("surv", C.c_void_p), ("cap", C.c_uint32),
                ("tr", C.c_uint32), ("ob", C.c_uint32), ("frame_len", C.c_int32),
                ("code_rate", C.c_int32), ("depth", C.c_int32)]


# ---------------------------------------------------------------- FFT / demap
def fft64(x):
    """x: int16 array [..., 64, 2] (re, im).  Returns the same shape."""
    x = np.ascontiguousarray(x, dtype=np.int16)
    flat = x.reshape(-1, 64, 2)
    out = np.empty_like(flat)
    L = lib()
    for i in range(flat.shape[0]):
        L.zo_fft64(_p(flat[i]), _p(out[i]))
    return out.reshape(x.shape)


FFT_SIZES = (12, 16, 24, 32, 36, 48, 60, 64, 72, 96, 108, 120, 128, 144, 180, 192, 216, 240, 256, 288, 300,
             324, 360, 384, 432, 480, 512, 540, 576, 600, 648, 720, 768, 864, 900, 960, 972, 1024, 1080, 1152,
             1200, 2048)                       # __ext_sora_fft's sizes (csrc/sora_ext_lib.cpp:2672-2812)


def fft_n(n, x):
    """FFTSafe<n> of every row: x int16 [..., n, 2].  Raises for a size the reference rejects."""
    x = np.ascontiguousarray(x, dtype=np.int16)
    flat = x.reshape(-1, n, 2)
    out = np.empty_like(flat)
    L = lib()
    for i in range(flat.shape[0]):
        if L.zo_fft_n(int(n), _p(flat[i]), _p(out[i])) != 0:
            raise ValueError(f"fft size {n} not supported")
    return out.reshape(x.shape)


def v_shift_right_complex16(x, shift):
    x = np.ascontiguousarray(x, dtype=np.int16).reshape(-1, 2)
    z = np.zeros_like(x)
    lib().zo_v_shift_right_complex16(_p(z), _p(x), x.shape[0], int(shift))
    return z


def get_data(f64):
    f64 = np.ascontiguousarray(f64, dtype=np.int16).reshape(64, 2)
    o = np.empty((48, 2), np.int16)
    lib().zo_get_data(_p(f64), _p(o))
    return o


def demap_limit(x):
    x = np.ascontiguousarray(x, dtype=np.int16).reshape(-1, 2)
    o = np.empty_like(x)
    lib().zo_demap_limit(_p(x), x.shape[0], _p(o))
    return o


def demap(mod, lim48):
    lim48 = np.ascontiguousarray(lim48, dtype=np.int16).reshape(48, 2)
    o = np.empty(288, np.int8)
    n = lib().zo_demap(mod, _p(lim48), _p(o))
    return o[:n]


def ncbps(mod):
    return lib().zo_ncbps(mod)


def ndbps(mod, coding):
    return lib().zo_ndbps(mod, coding)


def deinterleave(mod, soft):
    soft = np.ascontiguousarray(soft, dtype=np.int8)
    o = np.empty_like(soft)
    lib().zo_deinterleave(mod, _p(soft), _p(o))
    return o


def deint_perm(mod):
    return np.array([lib().zo_deint_src(mod, k) for k in range(ncbps(mod))], np.int32)


def luts():
    L = lib()
    return np.array([[L.zo_lut(w)[i] for i in range(256)] for w in range(4)], np.uint8)


def twiddle(N, k, n):
    re, im = C.c_int16(), C.c_int16()
    lib().zo_twiddle(N, k, n, C.byref(re), C.byref(im))
    return re.value, im.value


# ---------------------------------------------------------------- Viterbi
class Viterbi:
    """Stateful decoder with __ext_viterbi_brick_init_fast / _decode_fast semantics."""

    def __init__(self):
        self.v = Vit()

    def init(self, frame_len, code_rate, depth=256):
        lib().zo_vit_init(C.byref(self.v), frame_len, code_rate, depth)

    def decode(self, soft):
        soft = np.ascontiguousarray(soft, dtype=np.int8)
        out = np.zeros(4096 + 64, np.uint8)
        bits = lib().zo_vit_decode(C.byref(self.v), _p(soft), soft.size, _p(out))
        return out[: bits // 8].copy()

    def __del__(self):
        try:
            lib().zo_vit_free(C.byref(self.v))
        except Exception:
            pass


def viterbi_decode(soft, frame_len, code_rate, chunk=48):
    """init + feed all soft (in calls of `chunk` values) -> decoded bytes."""
    d = Viterbi()
    d.init(frame_len, code_rate)
    soft = np.asarray(soft, np.int8)
    outs = [d.decode(soft[i:i + chunk]) for i in range(0, soft.size, chunk)]
    return np.concatenate(outs) if outs else np.zeros(0, np.uint8)


def viterbi_sig(soft48):
    soft48 = np.ascontiguousarray(soft48, dtype=np.int8)
    o = np.zeros(4, np.uint8)
    lib().zo_vit_sig(_p(soft48), _p(o))
    return o


def vit_lut(which, soft, k, j):
    return lib().zo_vit_lut(which, soft, k, j)


def viterbi_batch(soft, soft_off, soft_len, frame_len, code_rate, out_off, out_size, nthreads=1, fast=False):
    """fast: the CPU port's AVX-512 brick loop (zp_viterbi_batch, bench.py's config-2
    cpu_baseline), identical output (tests/test_cpu_port.py)."""
    soft = np.ascontiguousarray(soft, np.int8)
    out = np.zeros(out_size, np.uint8)
    args = [np.ascontiguousarray(a, t) for a, t in
            ((soft_off, np.int64), (soft_len, np.int32), (frame_len, np.int32),
             (code_rate, np.int16), (out_off, np.int64))]
    fn = lib().zp_viterbi_batch if fast else lib().zo_viterbi_batch
    fn(_p(soft), _p(args[0]), _p(args[1]), _p(args[2]), _p(args[3]), len(args[0]), _p(out), _p(args[4]), nthreads)
    return out


# ---------------------------------------------------------------- header / CRC / chain
def parse_header(hb3):
    hb = np.zeros(4, np.uint8)
    hb[:3] = hb3[:3]
    h = (C.c_int32 * 4)()
    lib().zo_parse_header(_p(hb), h)
    return dict(coding=h[0], modulation=h[1], len=h[2], err=h[3])


def crc32_bits(b):
    b = np.ascontiguousarray(b, np.uint8)
    return lib().zo_crc32_bits(_p(b), b.size)


def descramble_crc(decoded, length):
    decoded = np.ascontiguousarray(decoded, np.uint8)
    pay = np.zeros(max(length, 4) + 8, np.uint8)
    ok = lib().zo_descramble_crc(_p(decoded), length, _p(pay))
    return pay[: max(length - 4, 0)].copy(), bool(ok)


def _res(r):
    return dict(coding=r.coding, modulation=r.modulation, len=r.len, err=r.err,
                crc_ok=r.crc_ok, nsym_used=r.nsym_used, viterbi_bits=r.viterbi_bits)


def rx_packet_freq(sub48):
    sub48 = np.ascontiguousarray(sub48, np.int16).reshape(-1, 48, 2)
    pay = np.zeros(4200, np.uint8)
    r = RxResult()
    ret = lib().zo_rx_packet_freq(_p(sub48), sub48.shape[0], _p(pay), C.byref(r))
    d = _res(r)
    d["ret"] = ret
    return pay[: max(d["len"] - 4, 0)].copy(), d


def rx_packet_time(sym):
    sym = np.ascontiguousarray(sym, np.int16).reshape(-1, 64, 2)
    pay = np.zeros(4200, np.uint8)
    r = RxResult()
    ret = lib().zo_rx_packet_time(_p(sym), sym.shape[0], _p(pay), C.byref(r))
    d = _res(r)
    d["ret"] = ret
    return pay[: max(d["len"] - 4, 0)].copy(), d


def rx_batch_time(sym, sym_off, nsym, payload_stride=4096, nthreads=1):
    """Full chain over packets; sym int16 [nsyms_total, 64, 2]; sym_off in symbols."""
    sym = np.ascontiguousarray(sym, np.int16)
    sym_off = np.ascontiguousarray(sym_off, np.int64)
    nsym = np.ascontiguousarray(nsym, np.int32)
    n = sym_off.size
    pay = np.zeros((n, payload_stride), np.uint8)
    res = (RxResult * n)()
    lib().zo_rx_batch_time(_p(sym), _p(sym_off), _p(nsym), n, _p(pay), payload_stride, res, nthreads)
    return pay, [_res(r) for r in res]


def rx_batch_time_fast(sym, sym_off, nsym, payload_stride=4096, nthreads=1):
    """rx_batch_time by the fast CPU port (oracle/cpu_port.c: table FFT, AVX-512 ACS, table
    CRC), bit-identical to it (tests/test_cpu_port.py); bench.py's cpu_baseline leg."""
    sym = np.ascontiguousarray(sym, np.int16)
    sym_off = np.ascontiguousarray(sym_off, np.int64)
    nsym = np.ascontiguousarray(nsym, np.int32)
    n = sym_off.size
    pay = np.zeros((n, payload_stride), np.uint8)
    res = (RxResult * n)()
    L = lib()
    L.zp_rx_batch_time.restype = C.c_int
    rx_batch_time_fast.avx512 = bool(L.zp_rx_batch_time(_p(sym), _p(sym_off), _p(nsym), n, _p(pay),
                                                        payload_stride, res, nthreads))
    return pay, [_res(r) for r in res]


# ---------------------------------------------------------------- synthetic TX
def tx_encode(bits, coding):
    bits = np.ascontiguousarray(bits, np.uint8)
    out = np.zeros(bits.size * 2, np.uint8)
    k = lib().zo_tx_encode(_p(bits), bits.size, coding, _p(out))
    return out[:k]


def tx_packet_freq(payload, mod, coding):
    """SIGNAL + data symbols in GetData order: int16 [nsym, 48, 2]."""
    payload = np.ascontiguousarray(payload, np.uint8)
    L = lib()
    maxs = 2 + (16 + 8 * payload.size + 38) // 24
    sub = np.zeros((1 + maxs, 48, 2), np.int16)
    L.zo_tx_signal_symbol(mod, coding, payload.size + 4, _p(sub[0]))
    n = L.zo_tx_data_symbols(_p(payload), payload.size, mod, coding, _p(sub[1:]), maxs)
    assert n > 0
    return sub[: 1 + n].copy()


# ---------------------------------------------------------------- ChannelEqualization + PilotTrack
def _fix_trig(L):
    for f in ("zo_sin16", "zo_cos16", "zo_atan2_16", "zo_trig_sin_entry", "zo_trig_cos_entry",
              "zo_trig_atan2_entry"):
        getattr(L, f).restype = C.c_int16
    return L


def trig_tables():
    """(sin, cos) over all 65536 unsigned angles and the atan2x table [256*256], int16."""
    L = _fix_trig(lib())
    s = np.array([L.zo_trig_sin_entry(r) for r in range(65536)], np.int16)
    c = np.array([L.zo_trig_cos_entry(r) for r in range(65536)], np.int16)
    a = np.array([L.zo_trig_atan2_entry(((i >> 8) & 255) - 256 * ((i >> 15) & 1), (i & 255) - 256 * ((i >> 7) & 1))
                  for i in range(65536)], np.int16)
    return s, c, a


def atan2_16(y, x):
    return _fix_trig(lib()).zo_atan2_16(C.c_int16(int(y)), C.c_int16(int(x)))


def v_mul_complex16(x, y, shift):
    x = np.ascontiguousarray(x, np.int16).reshape(-1, 2)
    y = np.ascontiguousarray(y, np.int16).reshape(-1, 2)
    o = np.zeros_like(x)
    lib().zo_v_mul_complex16(_p(o), _p(x), _p(y), x.shape[0], int(shift))
    return o


def channel_eq(sym64, coeffs64):
    s = np.ascontiguousarray(sym64, np.int16).reshape(64, 2)
    c = np.ascontiguousarray(coeffs64, np.int16).reshape(64, 2)
    o = np.zeros_like(s)
    lib().zo_channel_eq(_p(s), _p(c), _p(o))
    return o


def pilot_track(sym64, k):
    s = np.ascontiguousarray(sym64, np.int16).reshape(64, 2)
    o = np.zeros_like(s)
    lib().zo_pilot_track(_p(s), int(k), _p(o))
    return o


def ofdm_eq_symbol(sym64, coeffs64, k):
    s = np.ascontiguousarray(sym64, np.int16).reshape(64, 2)
    c = np.ascontiguousarray(coeffs64, np.int16).reshape(64, 2)
    o = np.zeros_like(s)
    lib().zo_ofdm_eq_symbol(_p(s), _p(c), int(k), _p(o))
    return o


def rx_batch_time_eq(sym, sym_off, nsym, chan, payload_stride=4096, nthreads=1):
    """receiver.blk:66-71 over packets: chan int16 [n, 64, 2] channel coefficients."""
    sym = np.ascontiguousarray(sym, np.int16)
    sym_off = np.ascontiguousarray(sym_off, np.int64)
    nsym = np.ascontiguousarray(nsym, np.int32)
    chan = np.ascontiguousarray(chan, np.int16)
    n = sym_off.size
    pay = np.zeros((n, payload_stride), np.uint8)
    res = (RxResult * n)()
    lib().zo_rx_batch_time_eq(_p(sym), _p(sym_off), _p(nsym), n, _p(chan), _p(pay), payload_stride, res,
                              nthreads)
    return pay, [_res(r) for r in res]



def rx_batch_time_eq_fast(sym, sym_off, nsym, chan, payload_stride=4096, nthreads=1):
    """rx_batch_time_eq by the fast CPU port (cpu_port.c: its FFT and Viterbi around the
    oracle's ChannelEqualization / PilotTrack), bit-identical (tests/test_cpu_port.py);
    bench.py --eq's cpu_baseline leg."""
    sym = np.ascontiguousarray(sym, np.int16)
    sym_off = np.ascontiguousarray(sym_off, np.int64)
    nsym = np.ascontiguousarray(nsym, np.int32)
    chan = np.ascontiguousarray(chan, np.int16)
    n = sym_off.size
    pay = np.zeros((n, payload_stride), np.uint8)
    res = (RxResult * n)()
    L = lib()
    L.zp_rx_batch_time_eq.restype = C.c_int
    rx_batch_time_eq_fast.avx512 = bool(L.zp_rx_batch_time_eq(_p(sym), _p(sym_off), _p(nsym), n, _p(chan), _p(pay),
                                                              payload_stride, res, nthreads))
    return pay, [_res(r) for r in res]


# ---------------------------------------------------------------- RX front end
class CCA(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("noSamples", "shift", "energy", "noise", "maxCorr")]


def ifft64(x):
    x = np.ascontiguousarray(x, np.int16).reshape(64, 2)
    o = np.zeros_like(x)
    lib().zo_ifft64(_p(x), _p(o))
    return o


def downsample(x):
    x = np.ascontiguousarray(x, np.int16).reshape(-1, 2)
    o = np.zeros_like(x)
    n = lib().zo_downsample(_p(x), x.shape[0], _p(o))
    return o[:n].copy()


def cca_pattern():
    o = np.zeros((256, 2), np.int16)
    lib().zo_cca_pattern(_p(o))
    return o


def lts_coeffs(xp144, shift, amp, sora_compat=False):
    xp = np.ascontiguousarray(xp144, np.int16).reshape(144, 2)
    o = np.zeros((64, 2), np.int16)
    lib().zo_lts_coeffs_mode(_p(xp), int(shift), int(amp), _p(o), 1 if sora_compat else 0)
    return o


def rx_stream(x):
    """receiver() on one stream (after any downSample): (payload, result dict, det dict,
    coeffs [64,2], data_start) or None when no packet is detected."""
    x = np.ascontiguousarray(x, np.int16).reshape(-1, 2)
    pay = np.zeros(4200, np.uint8)
    r, det, d0 = RxResult(), CCA(), C.c_int()
    co = np.zeros((64, 2), np.int16)
    ret = lib().zo_rx_stream(_p(x), x.shape[0], _p(pay), C.byref(r), C.byref(det), _p(co), C.byref(d0))
    d = _res(r)
    d["ret"] = ret
    dd = {k: getattr(det, k) for k, _ in CCA._fields_}
    return pay[: max(d["len"] - 4, 0)].copy(), d, dd, co, d0.value



# ---------------------------------------------------------------- TX chain
def ifft128(x):
    x = np.ascontiguousarray(x, np.int16).reshape(128, 2)
    o = np.zeros_like(x)
    lib().zo_ifft128(_p(x), _p(o))
    return o


def tx_preamble():
    o = np.zeros((640, 2), np.int16)
    lib().zo_tx_preamble(_p(o))
    return o


def tx_packet(inp):
    """transmitter() on one packet: 3 PLCP header bytes + payload -> int16 [n, 2] samples."""
    inp = np.ascontiguousarray(inp, np.uint8)
    out = np.zeros((640 + 160 * 1500, 2), np.int16)
    n = lib().zo_tx_packet(_p(inp), inp.size, _p(out), out.shape[0])
    assert n > 0, n
    return out[:n].copy()


def plcp_header(mod, coding, length):
    """The 3 air bytes of a PLCP header (RATE, LENGTH, parity, tail; parsePLCPHeader.blk)."""
    rate = {(0, 0): 0xB, (0, 2): 0xF, (1, 0): 0xA, (1, 2): 0xE, (2, 0): 0x9, (2, 2): 0xD,
            (3, 1): 0x8, (3, 2): 0xC}[(mod, coding)]
    h = rate | (length << 5)
    h |= (bin(h).count("1") & 1) << 17
    return np.array([h & 255, (h >> 8) & 255, (h >> 16) & 255], np.uint8)
