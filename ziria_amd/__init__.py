"""ziria_amd — MI355X (gfx950) engine for the data-parallel 802.11a RX decode hot path of
Ziria (FFT64 -> GetData -> DemapLimit -> Demap -> Deinterleave -> depuncture -> K=7 soft
Viterbi -> descramble -> CRC-32), batched over packets.

The compute lives in libziria_rx.so (hand-written HIP kernels, ziria_amd/csrc); this
package is the host-side mirror of the reference's external-brick interface
(lib/externals.blk) plus a batched engine over device-resident buffers.
"""
from ._lib import LIB_PATH, ZiriaRxError, lib  # noqa: F401
from .externals import (sora_fft, sora_fft_dynamic, v_shift_right_complex16,  # noqa: F401
                        viterbi_brick_decode_fast, viterbi_brick_init_fast,
                        viterbiSig11a_brick_decode_fast, viterbiSig11a_brick_init_fast,
                        sora_fft64_batch, viterbi_batch_decode, wifi_rx_batch, wifi_rx_eq_batch, wifi_rx_stream_batch, wifi_tx_batch,
                        set_devices, get_devices, node_stats, set_host_register)

__all__ = ["sora_fft", "sora_fft_dynamic", "viterbi_brick_init_fast", "viterbi_brick_decode_fast",
           "viterbiSig11a_brick_init_fast", "viterbiSig11a_brick_decode_fast",
           "v_shift_right_complex16", "sora_fft64_batch", "viterbi_batch_decode", "wifi_rx_batch",
           "wifi_rx_eq_batch", "wifi_rx_stream_batch", "wifi_tx_batch",
           "set_devices", "get_devices", "node_stats", "set_host_register",
           "ZiriaRxError", "lib", "LIB_PATH"]
