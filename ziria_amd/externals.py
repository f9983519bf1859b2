"""Python mirror of the reference's external bricks (lib/externals.blk:110, 199-217) and of
the batched counterparts, over numpy arrays.  Same names, argument meaning and return
values as the Ziria externals; every call runs the HIP engine in libziria_rx.so.

  sora_fft(inp)                          externals.blk:201  (csrc/sora_ext_lib.cpp:2672)
  viterbi_brick_init_fast(len, rate, d)  externals.blk:215  (csrc/sora_ext_viterbi.cpp:49)
  viterbi_brick_decode_fast(svalue)      externals.blk:216  (csrc/sora_ext_viterbi.cpp:67)
  viterbiSig11a_brick_decode_fast(sv)    externals.blk:217  (csrc/sora_ext_viterbi.cpp:177)
  v_shift_right_complex16(x, shift)      externals.blk:110  (csrc/sora_ext_lib.cpp:1979)
"""
import ctypes as C

import numpy as np

from ._lib import ZiriaRxError, lib

PAYLOAD_STRIDE = 4096
INFO_FIELDS = ("modulation", "coding", "len", "header_err", "crc_ok", "status", "symbols_used",
               "viterbi_bits")


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _c16(x, n=None):
    x = np.ascontiguousarray(x, dtype=np.int16)
    if x.ndim == 1:
        x = x.reshape(-1, 2)
    if n is not None and x.shape[-2] != n:
        raise ValueError(f"expected {n} complex16 values")
    return x


def sora_fft(inp):
    """FFT of arr complex16 (re/im int16 pairs, shape [N, 2]), N any size the reference
    dispatches (12..2048, csrc/sora_ext_lib.cpp:2672-2812).  For another size the reference
    prints an error and leaves the output untouched; here the untouched output is all zeros
    (the Ziria caller's fresh array)."""
    x = _c16(inp)
    out = np.zeros_like(x)
    lib().__ext_sora_fft(_p(out), x.shape[0], _p(x), x.shape[0])
    return out


def sora_fft_dynamic(nFFTSize, inp):
    x = _c16(inp)
    out = np.zeros_like(x)
    lib().__ext_sora_fft_dynamic(_p(out), x.shape[0], int(nFFTSize), _p(x), x.shape[0])
    return out


def viterbi_brick_init_fast(frame_length, code_rate, depth=256):
    return lib().__ext_viterbi_brick_init_fast(int(frame_length), int(code_rate), int(depth))


def viterbiSig11a_brick_init_fast(frame_length, code_rate, depth=256):
    return lib().__ext_viterbiSig11a_brick_init_fast(int(frame_length), int(code_rate), int(depth))


def viterbi_brick_decode_fast(svalue):
    """Feeds soft values (arr[48] int8 in the WiFi RX); returns (nbits, bytes appended)."""
    s = np.ascontiguousarray(svalue, dtype=np.int8)
    out = np.zeros(s.size + 512, np.uint8)
    nbits = lib().__ext_viterbi_brick_decode_fast(_p(s), s.size, _p(out), out.size * 8)
    return int(nbits), out[: max(int(nbits), 0) // 8].copy()


def viterbiSig11a_brick_decode_fast(svalue, bit=None):
    """48 soft values -> the 4-byte word the brick leaves (already >>6); bits 0..17 are the
    PLCP header bits (ViterbiSig11a.blk:37 zeroes 18..23)."""
    s = np.ascontiguousarray(svalue, dtype=np.int8)
    if s.size != 48:
        raise ValueError("SIGNAL decode takes 48 soft values")
    out = np.zeros(4, np.uint8) if bit is None else np.ascontiguousarray(bit, np.uint8).copy()
    lib().__ext_viterbiSig11a_brick_decode_fast(_p(s), 48, _p(out), 32)
    return out


def v_shift_right_complex16(x, shift):
    x = _c16(x)
    z = np.zeros_like(x)
    lib().__ext_v_shift_right_complex16(_p(z), x.shape[0], _p(x), x.shape[0], int(shift))
    return z


# ------------------------------------------------------------------ batched (host arrays)
def sora_fft64_batch(sym):
    """sym int16 [nsym, 64, 2] -> FFT of every symbol."""
    x = np.ascontiguousarray(sym, dtype=np.int16).reshape(-1, 64, 2)
    out = np.zeros_like(x)
    lib().__ext_sora_fft64_batch(_p(out), x.shape[0] * 64, _p(x), x.shape[0] * 64)
    return out


def viterbi_batch_decode(soft, pkt_soft_off, frame_len, code_rate, pkt_out_off=None):
    """Batched brick: packet i decodes soft[pkt_soft_off[i]:pkt_soft_off[i+1]].
    Returns (out bytes, out offsets)."""
    soft = np.ascontiguousarray(soft, np.int8)
    so = np.ascontiguousarray(pkt_soft_off, np.int32)
    fl = np.ascontiguousarray(frame_len, np.int32)
    cr = np.ascontiguousarray(code_rate, np.int16)
    n = so.size - 1
    if pkt_out_off is None:
        pkt_out_off = (np.cumsum(fl) - fl).astype(np.int32)
    oo = np.ascontiguousarray(pkt_out_off, np.int32)
    total = int((oo + fl).max()) if n > 0 else 0
    out = np.zeros(max(total, 1), np.uint8)
    rc = lib().__ext_viterbi_batch_decode(_p(soft), soft.size, _p(so), so.size, _p(fl), n, _p(cr), n,
                                          _p(out), out.size * 8, _p(oo), n)
    if rc < 0:
        raise ZiriaRxError(f"__ext_viterbi_batch_decode failed ({rc})")
    return out, oo


def wifi_rx_batch(sym, pkt_sym_off):
    """Batched receiveBits over time-domain packets.  sym int16 [S, 64, 2]; pkt_sym_off
    (n+1) CSR symbol offsets.  Returns (payload uint8 [n, 4096], info dict of arrays, crc
    pass count)."""
    x = np.ascontiguousarray(sym, dtype=np.int16).reshape(-1, 64, 2)
    off = np.ascontiguousarray(pkt_sym_off, np.int32)
    n = off.size - 1
    pay = np.zeros((max(n, 1), PAYLOAD_STRIDE), np.uint8)
    info = np.zeros((max(n, 1), 8), np.int32)
    rc = lib().__ext_wifi_rx_batch(_p(x), x.shape[0], _p(off), off.size, _p(pay), pay.size * 8,
                                   _p(info), info.size)
    if rc < 0:
        raise ZiriaRxError(f"__ext_wifi_rx_batch failed ({rc})")
    return pay[:n], {k: info[:n, i].copy() for i, k in enumerate(INFO_FIELDS)}, int(rc)


def wifi_rx_eq_batch(sym, pkt_sym_off, chan):
    """wifi_rx_batch with ChannelEqualization + PilotTrack (receiver.blk:66-71); chan int16
    [n, 64, 2]: each packet's LTS channel coefficients."""
    x = np.ascontiguousarray(sym, dtype=np.int16).reshape(-1, 64, 2)
    off = np.ascontiguousarray(pkt_sym_off, np.int32)
    ch = np.ascontiguousarray(chan, np.int16).reshape(-1, 64, 2)
    n = off.size - 1
    pay = np.zeros((max(n, 1), PAYLOAD_STRIDE), np.uint8)
    info = np.zeros((max(n, 1), 8), np.int32)
    rc = lib().__ext_wifi_rx_eq_batch(_p(x), x.shape[0], _p(off), off.size, _p(ch), ch.shape[0] * 64,
                                      _p(pay), pay.size * 8, _p(info), info.size)
    if rc < 0:
        raise ZiriaRxError(f"__ext_wifi_rx_eq_batch failed ({rc})")
    return pay[:n], {k: info[:n, i].copy() for i, k in enumerate(INFO_FIELDS)}, int(rc)


def wifi_rx_stream_batch(samples, cap_off, downsample=False):
    """receiver() once per capture (receiver.blk:57-72) over host arrays: samples int16
    [S, 2]; cap_off (n+1) CSR sample offsets.  Returns (payload uint8 [n, 4096], info dict,
    det int32 [n, 8], count of detected packets whose CRC passed)."""
    x = np.ascontiguousarray(samples, dtype=np.int16).reshape(-1, 2)
    off = np.ascontiguousarray(cap_off, np.int32)
    n = off.size - 1
    pay = np.zeros((max(n, 1), PAYLOAD_STRIDE), np.uint8)
    info = np.zeros((max(n, 1), 8), np.int32)
    det = np.zeros((max(n, 1), 8), np.int32)
    rc = lib().__ext_wifi_rx_stream_batch(_p(x), x.shape[0], _p(off), off.size, 1 if downsample else 0,
                                          _p(pay), pay.size * 8, _p(info), info.size, _p(det), det.size)
    if rc < 0:
        raise ZiriaRxError(f"__ext_wifi_rx_stream_batch failed ({rc})")
    return pay[:n], {k: info[:n, i].copy() for i, k in enumerate(INFO_FIELDS)}, det[:n], int(rc)


def wifi_tx_batch(packets):
    """transmitter() per packet (transmitter.blk at 40 MHz): packets = list of uint8 arrays,
    each 3 PLCP header bytes + payload.  Returns (samples int16 [S, 2], offsets int32 [n+1])."""
    data = np.concatenate([np.asarray(p, np.uint8) for p in packets]) if packets else np.zeros(0, np.uint8)
    ioff = np.cumsum([0] + [len(p) for p in packets]).astype(np.int32)
    n = len(packets)
    total = sum(int(lib().zrx_tx_samples(_p(np.ascontiguousarray(np.asarray(p, np.uint8)[:3])))) for p in packets)
    out = np.zeros((max(total, 1), 2), np.int16)
    ooff = np.zeros(n + 1, np.int32)
    rc = lib().__ext_wifi_tx_batch(_p(np.ascontiguousarray(data)), data.size, _p(ioff), n + 1, _p(out),
                                   out.shape[0], _p(ooff), n + 1)
    if rc < 0:
        raise ZiriaRxError(f"__ext_wifi_tx_batch failed ({rc})")
    return out[:total], ooff


# ------------------------------------------------------------------ the node behind Part 2
def set_devices(devices=None, min_shard_bytes=-1):
    """Logical shards of the batched externals (zrx_set_devices): a list of device ids (a
    device may repeat), or None for the default (ZRX_DEVICES, else every gfx950 device);
    min_shard_bytes < 0 keeps the default 16 MiB, 0 spreads every call over every shard."""
    d = np.ascontiguousarray(devices if devices is not None else [], np.int32)
    rc = lib().zrx_set_devices(_p(d) if d.size else None, int(d.size), int(min_shard_bytes))
    if rc < 0:
        raise ZiriaRxError(f"zrx_set_devices failed ({rc})")


def get_devices():
    d = np.zeros(64, np.int32)
    n = lib().zrx_get_devices(_p(d), d.size)
    if n < 0:
        raise ZiriaRxError(f"zrx_get_devices failed ({n})")
    return [int(x) for x in d[:n]]


NODE_STATS = ("last_shards", "register_mode", "registered_ranges", "registered_bytes", "registrations",
              "register_hits", "register_failures", "min_shard_bytes")


def node_stats():
    s = np.zeros(8, np.int64)
    lib().zrx_node_stats(_p(s))
    return dict(zip(NODE_STATS, (int(x) for x in s)))


def set_host_register(mode):
    """0 = never page-lock caller arrays, 1 = the main program's static arrays (default), 2 =
    also other arrays >= 32 KiB (the caller keeps them mapped until mode 0 or 1)."""
    rc = lib().zrx_set_host_register(int(mode))
    if rc < 0:
        raise ZiriaRxError(f"zrx_set_host_register failed ({rc})")
