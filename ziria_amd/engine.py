"""Batched decode engine over device-resident (HBM) buffers.

Drives the Part-3 C-ABI of libziria_rx.so (zrx_*) with torch tensors as the device memory
allocator and torch's current HIP stream as the launch stream; torch is plumbing here, the
kernels are the hand-written HIP in ziria_amd/csrc.
"""
import ctypes as C

import torch

from ._lib import ZiriaRxError, check, lib

PAYLOAD_STRIDE = 4096
STAGES = ("signal_fft", "signal_viterbi", "data_fft_demap", "data_viterbi", "descramble_crc")


def _ptr(t):
    return C.c_void_p(t.data_ptr())


class RxEngine:
    """One engine context per device.  Methods launch asynchronously on the current stream."""

    def __init__(self, device=0):
        if not torch.cuda.is_available():
            raise ZiriaRxError("RxEngine needs a HIP device (no CPU path)")
        self.device = torch.device("cuda", device)
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device).cuda_stream
            check(lib().zrx_create(C.byref(h), device, C.c_void_p(stream)), "zrx_create")
        self._h = h

    def close(self):
        if self._h:
            lib().zrx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        s = torch.cuda.current_stream(self.device).cuda_stream
        check(lib().zrx_set_stream(self._h, C.c_void_p(s)), "zrx_set_stream")

    def reserve(self, npkts, max_nsym):
        check(lib().zrx_reserve(self._h, int(npkts), int(max_nsym)), "zrx_reserve")

    def enable_timing(self, on=True):
        check(lib().zrx_enable_timing(self._h, 1 if on else 0), "zrx_enable_timing")

    def stage_ms(self):
        ms = (C.c_float * 5)()
        check(lib().zrx_get_timing(self._h, ms), "zrx_get_timing")
        return dict(zip(STAGES, [float(v) for v in ms]))

    def plan_stats(self):
        """(decoder rows, frames re-decoded by the seam pass) of the last Viterbi launch."""
        st = (C.c_int32 * 2)()
        check(lib().zrx_plan_stats(self._h, st), "zrx_plan_stats")
        return int(st[0]), int(st[1])

    def plan_check(self):
        """Raises if the last Viterbi plan dropped rows past its workspace bound (ZRX_EPLAN)."""
        check(lib().zrx_plan_check(self._h), "zrx_plan_check")

    def link(self, other, mode):
        """Two engines taking a stream of batches in turn (zrx_pipeline_link): mode bit 0 =
        this engine's data Viterbi waits for the other's last launched chain, bit 1 = its data
        FFT waits for the other's last launched Viterbi, bit 2 = its chain's head (SIGNAL,
        plan, data FFT) on a lowest-priority stream; 0 unlinks."""
        check(lib().zrx_pipeline_link(self._h, other._h, int(mode)), "zrx_pipeline_link")

    # ------------------------------------------------------------------ launches
    def fft64(self, sym, out=None):
        """sym: int16 [S, 64, 2] on the device -> FFT64 of every symbol."""
        assert sym.dtype == torch.int16 and sym.is_contiguous() and sym.shape[-2:] == (64, 2)
        out = torch.empty_like(sym) if out is None else out
        self._stream()
        check(lib().zrx_fft64_dev(self._h, _ptr(sym), _ptr(out), sym.numel() // 128), "zrx_fft64_dev")
        return out

    def fft(self, n, x, out=None):
        """FFTSafe<n> of every row: x int16 [..., n, 2] on the device (n any __ext_sora_fft
        size, 12..2048)."""
        assert x.dtype == torch.int16 and x.is_contiguous() and x.shape[-2:] == (n, 2)
        out = torch.empty_like(x) if out is None else out
        self._stream()
        check(lib().zrx_fft_dev(self._h, int(n), _ptr(x), _ptr(out), x.numel() // (2 * n)), "zrx_fft_dev")
        return out

    def viterbi(self, soft, soft_off, params, out, out_off, out_bits):
        """soft int8, soft_off int64 [n], params int32 [n,4] {frame_len, code_rate,
        soft_len, 0}, out uint8, out_off int64 [n], out_bits int32 [n] (all on device)."""
        n = soft_off.numel()
        for t in (soft, soft_off, params, out, out_off, out_bits):
            assert t.is_cuda and t.is_contiguous()
        assert params.dtype == torch.int32 and params.numel() == 4 * n
        self._stream()
        check(lib().zrx_viterbi_dev(self._h, _ptr(soft), _ptr(soft_off), _ptr(params), n, _ptr(out),
                                    _ptr(out_off), _ptr(out_bits)), "zrx_viterbi_dev")

    def rx(self, sym, sym_off, nsym, max_nsym, payload=None, info=None, chan=None):
        """Full chain.  sym int16 [S,64,2]; sym_off int64 [n] (SIGNAL symbol index);
        nsym int32 [n].  With chan (int16 [n,64,2], each packet's LTS channel coefficients)
        ChannelEqualization + PilotTrack run between FFT and GetData (receiver.blk:66-71).
        Returns (payload uint8 [n,4096], info int32 [n,8])."""
        n = sym_off.numel()
        assert sym.dtype == torch.int16 and sym_off.dtype == torch.int64 and nsym.dtype == torch.int32
        if payload is None:
            payload = torch.zeros((n, PAYLOAD_STRIDE), dtype=torch.uint8, device=sym.device)
        if info is None:
            info = torch.zeros((n, 8), dtype=torch.int32, device=sym.device)
        self._stream()
        if chan is None:
            check(lib().zrx_rx_dev(self._h, _ptr(sym), _ptr(sym_off), _ptr(nsym), n, int(max_nsym),
                                   _ptr(payload), _ptr(info)), "zrx_rx_dev")
        else:
            assert chan.dtype == torch.int16 and chan.is_contiguous() and chan.numel() == 128 * n
            check(lib().zrx_rx_eq_dev(self._h, _ptr(sym), _ptr(sym_off), _ptr(nsym), n, int(max_nsym),
                                      _ptr(chan), _ptr(payload), _ptr(info)), "zrx_rx_eq_dev")
        return payload, info

    def ofdm_eq(self, sym, sym_off, nsym, chan, out=None):
        """FFT >>> ChannelEqualization >>> PilotTrack of every symbol of every packet
        (PilotTrack's full 64-bin output, same layout as sym)."""
        n = sym_off.numel()
        assert sym.dtype == torch.int16 and chan.dtype == torch.int16 and chan.numel() == 128 * n
        out = torch.zeros_like(sym) if out is None else out
        self._stream()
        check(lib().zrx_ofdm_eq_dev(self._h, _ptr(sym), _ptr(sym_off), _ptr(nsym), n, _ptr(chan), _ptr(out)),
              "zrx_ofdm_eq_dev")
        return out

    def rx_stream(self, samples, cap_off, cap_len, max_len, downsample=False, payload=None, info=None, det=None):
        """receiver() (receiver.blk:57-72) once per capture: samples int16 [S, 2] on the device,
        cap_off int64 / cap_len int32 [n] in samples.  Returns (payload uint8 [n,4096], info
        int32 [n,8], det int32 [n,8] = {detected, noSamples, shift, energy, noise, maxCorr,
        consumed, data_start})."""
        n = cap_off.numel()
        assert samples.dtype == torch.int16 and cap_off.dtype == torch.int64 and cap_len.dtype == torch.int32
        dev = samples.device
        payload = torch.zeros((n, PAYLOAD_STRIDE), dtype=torch.uint8, device=dev) if payload is None else payload
        info = torch.zeros((n, 8), dtype=torch.int32, device=dev) if info is None else info
        det = torch.zeros((n, 8), dtype=torch.int32, device=dev) if det is None else det
        self._stream()
        check(lib().zrx_rx_stream_dev(self._h, _ptr(samples), _ptr(cap_off), _ptr(cap_len), n, int(max_len),
                                      1 if downsample else 0, _ptr(payload), _ptr(info), _ptr(det)),
              "zrx_rx_stream_dev")
        return payload, info, det
