// The externals of include/ziria_rx.h Parts 1 and 2 with C++ linkage: the symbols a
// wplc-compiled WiFi receiver links against.  wplc emits `fun external` prototypes into
// test.cpp (src/Codegen/CgFun.hs:287-316) and the reference builds every source with g++
// (csrc/Makefile:92-96), so the program references mangled names over the reference's types
// (num8 = char, int16 = short, int32 = int): e.g. _Z31__ext_viterbi_brick_decode_fastPciPhi,
// the name `nm` shows on the reference's own sora_ext_viterbi.o.  This translation unit
// includes the header as a C++ includer does and defines those declarations; each forwards
// to the implementation the C-linkage export uses (zrx_host.cpp: per-call, host CPU;
// zrx_api.hip: batched, GPU).
#include "../../include/ziria_rx.h"
#include "zrx_internal.h"

// ---- Part 1: per-call (csrc/sora_ext_lib.cpp:1979,2672,2818; csrc/sora_ext_viterbi.cpp:49,67,159,177)
void __ext_sora_fft(struct complex16* out, int nFFTSize, struct complex16* in, int unused1) {
  (void)unused1;
  zrx_host::sora_fft(out, nFFTSize, in);
}
void __ext_sora_fft_dynamic(struct complex16* out, int unused2, int16_t nFFTSize, struct complex16* in, int unused1) {
  (void)unused2;
  __ext_sora_fft(out, nFFTSize, in, unused1);
}
int __ext_viterbi_brick_init_fast(int32_t frame_len, int16_t code_rate, int16_t depth) {
  return zrx_host::vit_init(frame_len, code_rate, depth);
}
int16_t __ext_viterbi_brick_decode_fast(char* intInput, int len1, unsigned char* bit, int len2) {
  (void)len2;
  return zrx_host::vit_decode(intInput, len1, bit);
}
int __ext_viterbiSig11a_brick_init_fast(int32_t frame_len, int16_t code_rate, int16_t depth) {
  return zrx_host::vit_init(frame_len, code_rate, depth);
}
int16_t __ext_viterbiSig11a_brick_decode_fast(char* intInput, int len1, unsigned char* bit, int len2) {
  (void)len1; (void)len2;
  zrx_host::sig_decode(intInput, bit);
  return 0;
}
int __ext_v_shift_right_complex16(struct complex16* z, int unused3, struct complex16* x, int len, int shift) {
  (void)unused3;
  return zrx_host::shift_right(z, x, len, shift);
}

// ---- Part 2: batched (GPU)
void __ext_sora_fft64_batch(struct complex16* out, int outlen, struct complex16* in, int inlen) {
  zrx_batch::sora_fft64_batch(out, outlen, in, inlen);
}
int32_t __ext_viterbi_batch_decode(char* soft, int softlen, int32_t* pkt_soft_off, int n_off, int32_t* frame_len,
                                   int n_fl, int16_t* code_rate, int n_cr, unsigned char* out_bits,
                                   int out_len_bits, int32_t* pkt_out_off, int n_oo) {
  return zrx_batch::viterbi_batch_decode(soft, softlen, pkt_soft_off, n_off, frame_len, n_fl, code_rate, n_cr,
                                         out_bits, out_len_bits, pkt_out_off, n_oo);
}
int32_t __ext_wifi_rx_batch(struct complex16* sym, int nsym_total, int32_t* pkt_sym_off, int n_off,
                            unsigned char* payload, int payload_len_bits, int32_t* pkt_info, int n_info) {
  return zrx_batch::wifi_rx_batch(sym, nsym_total, pkt_sym_off, n_off, nullptr, 0, payload, payload_len_bits,
                                  pkt_info, n_info);
}
int32_t __ext_wifi_rx_eq_batch(struct complex16* sym, int nsym_total, int32_t* pkt_sym_off, int n_off,
                               struct complex16* chan, int chan_len, unsigned char* payload, int payload_len_bits,
                               int32_t* pkt_info, int n_info) {
  if (!chan) return ZRX_EINVAL;
  return zrx_batch::wifi_rx_batch(sym, nsym_total, pkt_sym_off, n_off, chan, chan_len, payload, payload_len_bits,
                                  pkt_info, n_info);
}
int32_t __ext_wifi_rx_stream_batch(struct complex16* samples, int nsamples, int32_t* cap_off, int n_off,
                                   int downsample, unsigned char* payload, int payload_len_bits, int32_t* pkt_info,
                                   int n_info, int32_t* det, int n_det) {
  return zrx_batch::wifi_rx_stream_batch(samples, nsamples, cap_off, n_off, downsample, payload, payload_len_bits,
                                         pkt_info, n_info, det, n_det);
}
int32_t __ext_wifi_tx_batch(unsigned char* in, int inlen, int32_t* pkt_in_off, int n_off, struct complex16* out,
                            int outlen, int32_t* pkt_out_off, int n_oo) {
  return zrx_batch::wifi_tx_batch(in, inlen, pkt_in_off, n_off, out, outlen, pkt_out_off, n_oo);
}
