// Internal entry points of libziria_rx.so shared by its translation units (hidden: not part
// of the C-ABI).  The exported externals of include/ziria_rx.h exist twice, with C linkage
// (ctypes, C callers; zrx_host.cpp and zrx_api.hip) and with the C++ linkage a
// wplc-generated test.cpp links against (zrx_ext_cxx.cpp); both forward here.
//   zrx_host::  the per-call externals on the host CPU (zrx_host.cpp): SURVEY.md §8(b) item 1,
//               "a CPU path, with the GPU used only if batched"
//   zrx_batch:: the batched externals over host arrays, on the GPU (zrx_api.hip)
#pragma once
#include <stdint.h>

struct complex16;

#define ZRX_HIDDEN __attribute__((visibility("hidden")))

namespace zrx_host {
ZRX_HIDDEN void sora_fft(struct complex16* out, int nfft, const struct complex16* in);
ZRX_HIDDEN int vit_init(int32_t frame_len, int16_t code_rate, int16_t depth);
ZRX_HIDDEN int16_t vit_decode(const char* soft, int len, unsigned char* bit);
ZRX_HIDDEN void sig_decode(const char* soft48, unsigned char* bit);
ZRX_HIDDEN int shift_right(struct complex16* z, const struct complex16* x, int len, int shift);
}  // namespace zrx_host

namespace zrx_batch {
ZRX_HIDDEN void sora_fft64_batch(struct complex16* out, int outlen, struct complex16* in, int inlen);
ZRX_HIDDEN int32_t viterbi_batch_decode(const char* soft, int softlen, const int32_t* pkt_soft_off, int n_off,
                                        const int32_t* frame_len, int n_fl, const int16_t* code_rate, int n_cr,
                                        unsigned char* out_bits, int out_len_bits, const int32_t* pkt_out_off,
                                        int n_oo);
ZRX_HIDDEN int32_t wifi_rx_batch(struct complex16* sym, int nsym_total, const int32_t* pkt_sym_off, int n_off,
                                 const struct complex16* chan, int chan_len, unsigned char* payload,
                                 int payload_len_bits, int32_t* pkt_info, int n_info);
ZRX_HIDDEN int32_t wifi_rx_stream_batch(struct complex16* samples, int nsamples, const int32_t* cap_off, int n_off,
                                        int downsample, unsigned char* payload, int payload_len_bits,
                                        int32_t* pkt_info, int n_info, int32_t* det, int n_det);
ZRX_HIDDEN int32_t wifi_tx_batch(const unsigned char* in, int inlen, const int32_t* pkt_in_off, int n_off,
                                 struct complex16* out, int outlen, int32_t* pkt_out_off, int n_oo);
}  // namespace zrx_batch
