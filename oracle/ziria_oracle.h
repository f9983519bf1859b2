/*
 * ORACLE — test infrastructure only.
 *
 * Scalar C restatement of the Ziria 802.11a RX decode hot path, used (a) by tests/ as the
 * parity checker for the HIP engine, (b) by bench.py's cpu_baseline leg, (c) by
 * __graft_entry__.smoke() as the checker.  It is never linked into, loaded by, or called
 * from the product library (ziria_amd/).  Pinned against the reference's own KATs and
 * golden fixtures generated from the reference bricks (tests/golden/, see
 * tests/golden/make_golden.py) — see DESIGN.md "Oracle".
 *
 * Every function cites the reference file:line it restates (paths relative to the
 * moxfun/Ziria root).
 */
#ifndef ZIRIA_ORACLE_H
#define ZIRIA_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { int16_t re, im; } zo_c16;

/* ---- FFT64: csrc/fft_r4difx.hpp:54-140,220-237, csrc/sora_ext_lib_fft.hpp:41-108 ---- */
void zo_fft64(const zo_c16* in, zo_c16* out);
/* FFTSafe<N> for every size __ext_sora_fft dispatches (12..2048); -1 for others */
int zo_fft_n(int N, const zo_c16* in, zo_c16* out);
int zo_fft_supported(int N);
int zo_fft_radix(int N);
void zo_fft_freq_of_pos(int N, int* idx);
/* twiddles twFFTLUT{N}_{k} (csrc/sora_ext_lib_fft_coeffs.hpp:53-78,298-359) regenerated */
void zo_twiddle(int N, int k, int n, int16_t* re, int16_t* im);

int  zo_v_shift_right_complex16(zo_c16* z, const zo_c16* x, int len, int shift);  /* sora_ext_lib.cpp:1979 */

/* ---- GetData / DemapLimit / Demap* / Deinterleave* (code/WiFi/receiver/...) ---- */
void zo_get_data(const zo_c16* sym64, zo_c16* out48);            /* OFDM/GetData.blk:24-35 */
void zo_demap_limit(const zo_c16* in, int n, zo_c16* out);        /* decoding/DemapLimit.blk:22-63 */
int  zo_demap(int mod, const zo_c16* lim48, int8_t* soft);       /* decoding/Demap*.blk:22-33 */
int  zo_ncbps(int mod);                                          /* 48,96,192,288 */
int  zo_ndbps(int mod, int coding);                              /* transmitter.blk:39-46 */
int  zo_deint_src(int mod, int k);                               /* Deinterleave*.blk tables */
void zo_deinterleave(int mod, const int8_t* in, int8_t* out);
const uint8_t* zo_lut(int which);     /* 0 bpsk,1 qam16_2,2 qam64_2,3 qam64_3 (const.blk:74-150) */

/* ---- Viterbi brick: csrc/sora_ext_viterbi.cpp:38-153, csrc/viterbicore.hpp:98-399 ---- */
typedef struct {
  uint8_t  m[64];        /* current column metrics (u8, LSB = survivor marker) */
  uint64_t* surv;        /* survivor LSB word per column, column 0 = init */
  uint32_t cap;          /* columns allocated */
  uint32_t tr;           /* trellis index (columns after column 0) */
  uint32_t ob;           /* ob_count */
  int32_t  frame_len;    /* bytes to decode */
  int32_t  code_rate;    /* CR_12=0, CR_23=1, CR_34=2 */
  int32_t  depth;        /* TRELLIS_DEPTH (256 in the WiFi RX) */
} zo_vit;
int  zo_vit_init(zo_vit* v, int frame_len, int code_rate, int depth);
void zo_vit_free(zo_vit* v);
/* feeds n soft values (one or more whole groups); appends decoded bytes to out; returns bits */
int  zo_vit_decode(zo_vit* v, const int8_t* soft, int n, uint8_t* out);
/* SIGNAL: 48 soft -> 4 bytes as the brick leaves them (after the >>6 of :191) */
void zo_vit_sig(const int8_t* soft48, uint8_t* bits4);
/* branch metric as in VIT_MA / VIT_MB (csrc/viterbilut.h:111-285) */
int  zo_vit_lut(int which, int soft, int k, int j);

/* ---- PLCP header, descrambler, CRC (code/WiFi/transmitter/ .blk files) ---- */
typedef struct { int32_t coding, modulation, len, err; } zo_hdr;   /* const.blk:63-68 */
void zo_parse_header(const uint8_t* hbits3, zo_hdr* h);           /* parsePLCPHeader.blk:119-213 */
uint32_t zo_crc32_bits(const uint8_t* bytes, int nbytes);         /* crc.blk:41-73 bitwise */
/* Decode.blk:36-43 + crc_template.blk / check_crc (crc.blk:85-118):
   decoded = (len+2) bytes from the Viterbi; writes len-4 payload bytes; returns crc ok */
int  zo_descramble_crc(const uint8_t* decoded, int len, uint8_t* payload);

/* ---- full receive of one packet (receiver.blk:43-54 receiveBits, after GetData) ----
   sym: time-domain CP-removed symbols (64 complex16 each) starting with SIGNAL; nsym
   available.  Returns 0 ok, <0 if not enough symbols.  payload must hold 4096 bytes. */
typedef struct { zo_hdr h; int32_t crc_ok; int32_t nsym_used; int32_t viterbi_bits; } zo_rx_result;
int zo_rx_packet_time(const zo_c16* sym, int nsym, uint8_t* payload, zo_rx_result* r);
/* The same chain by the fast CPU port (cpu_port.c; bench.py's cpu_baseline only), identical
   results to zo_rx_batch_time; returns 1 when its AVX-512 Viterbi ran. */
int zp_fft64(const zo_c16* in, zo_c16* out, int n);
int zp_viterbi_batch(const int8_t* soft, const int64_t* soft_off, const int32_t* soft_len,
                     const int32_t* frame_len, const int16_t* code_rate, int npkts,
                     uint8_t* out, const int64_t* out_off, int nthreads);
int zp_rx_batch_time(const zo_c16* sym, const int64_t* sym_off, const int32_t* nsym, int npkts,
                     uint8_t* payload, int payload_stride, zo_rx_result* res, int nthreads);
int zp_rx_batch_time_eq(const zo_c16* sym, const int64_t* sym_off, const int32_t* nsym, int npkts, const zo_c16* chan,
                        uint8_t* payload, int payload_stride, zo_rx_result* res, int nthreads);
/* same, fed frequency-domain data subcarriers (48 per symbol, GetData order) */
int zo_rx_packet_freq(const zo_c16* sub48, int nsym, uint8_t* payload, zo_rx_result* r);

/* ---- ChannelEqualization + PilotTrack, ziria_oracle_eq.c ---- */
/* integer trigonometry (csrc/intalgx.h:38-99 over the LUTs of csrc/intalglutx.h) */
int16_t zo_sin16(int16_t r);                       /* sinx: FP_RAD, pi = 0x8000 */
int16_t zo_cos16(int16_t r);                       /* cosx */
int16_t zo_atan2_16(int16_t y, int16_t x);         /* atan2x */
int16_t zo_trig_sin_entry(int r);                  /* table entries, for the table checks */
int16_t zo_trig_cos_entry(int r);
int16_t zo_trig_atan2_entry(int yy, int xx);
int zo_pilot_sign(int m);                          /* pilotSgn[m] (PilotTrack.blk:70-78) */
/* __ext_v_mul_complex16 (sora_ext_lib.cpp:2098-2137) */
void zo_v_mul_complex16(zo_c16* out, const zo_c16* x, const zo_c16* y, int len, int shift);
/* ChannelEqualization.blk:26-46: bins 0..27, 36..63 times coeffs >> norm_shift (8) */
void zo_channel_eq(const zo_c16* in64, const zo_c16* coeffs64, zo_c16* out64);
/* PilotTrack.blk:56-249 on the k-th symbol of a packet (k = 0: the SIGNAL symbol) */
void zo_pilot_track(const zo_c16* in64, int k, zo_c16* out64);
/* FFT >>> ChannelEqualization >>> PilotTrack (receiver.blk:66-69) */
void zo_ofdm_eq_symbol(const zo_c16* sym64, const zo_c16* chan64, int k, zo_c16* out64);
/* receiver.blk:66-71 on one packet / a batch (chan: 64 coefficients per packet) */
int zo_rx_packet_time_eq(const zo_c16* sym, int nsym, const zo_c16* chan64, uint8_t* payload, zo_rx_result* r);
int zo_rx_batch_time_eq(const zo_c16* sym, const int64_t* sym_off, const int32_t* nsym, int npkts,
                        const zo_c16* chan, uint8_t* payload, int payload_stride, zo_rx_result* res,
                        int nthreads);

/* ---- RX front end, ziria_oracle_fe.c ---- */
typedef struct { int32_t noSamples; int32_t shift; int32_t energy; int32_t noise; int32_t maxCorr; } zo_cca;  /* const.blk:51-57 */
void zo_ifft64(const zo_c16* in, zo_c16* out);                     /* IFFT<64>, csrc/ifft_r4difx.hpp */
int  zo_downsample(const zo_c16* in, int n, zo_c16* out);          /* downSample.blk: returns n/8*4 */
void zo_cca_pattern(zo_c16* pattern256);                           /* cca_tufv.blk:50-98 */
int  zo_remove_dc(const zo_c16* x, int n, zo_c16* y);              /* removeDC.blk:25-85 */
/* removeDC >>> cca(threshold) (receiver.blk:38-40); 0 = detected */
int  zo_detect_preamble(const zo_c16* x, int n, int32_t energy_threshold, zo_cca* det, int* consumed);
int  zo_lts_agc_shift(int32_t amp);                                /* LTS.blk:146 */
void zo_lts_coeffs(const zo_c16* xp144, int shift, int32_t amp, zo_c16* coeffs64);   /* LTS.blk:113-203 */
void zo_lts_coeffs_mode(const zo_c16* xp144, int shift, int32_t amp, zo_c16* coeffs64, int sora_compat);
/* receiver() (receiver.blk:57-72) on one stream */
int  zo_rx_stream(const zo_c16* x, int n, uint8_t* payload, zo_rx_result* r, zo_cca* det, zo_c16* coeffs64,
                  int* data_start);

/* Batched Viterbi over packets (same semantics per packet as init + decode of all soft). */
int zo_viterbi_batch(const int8_t* soft, const int64_t* soft_off, const int32_t* soft_len,
                     const int32_t* frame_len, const int16_t* code_rate, int npkts,
                     uint8_t* out, const int64_t* out_off, int nthreads);
/* Batched full chain over packets, std pthreads over nthreads. */
int zo_rx_batch_time(const zo_c16* sym, const int64_t* sym_off, const int32_t* nsym, int npkts,
                     uint8_t* payload, int payload_stride, zo_rx_result* res, int nthreads);

/* ---- synthetic TX (test workload generator restating transmitter.blk:56-101) ---- */
/* bits (LSB-first bytes) of SERVICE+payload+CRC+pad, scrambled, encoded, punctured,
   interleaved, mapped: returns number of data symbols; writes 48 complex16 per symbol
   (GetData order) to sub48 (needs nsym*48 entries). */
int zo_tx_data_symbols(const uint8_t* payload, int len_minus4, int mod, int coding,
                       zo_c16* sub48, int max_sym);
int zo_tx_signal_symbol(int mod, int coding, int len, zo_c16* sub48);
int zo_tx_encode(const uint8_t* bits, int nbits, int coding, uint8_t* coded);  /* encoding.blk */
int zo_tx_signal_from_bits(const uint8_t* hbits3, zo_c16* sub48);              /* emitHeader >>> encode12 .. */
/* TX chain at 40 MHz, ziria_oracle_fe.c */
void zo_ifft128(const zo_c16* in, zo_c16* out);                    /* IFFT<128>, ifft_r4difx.hpp */
void zo_tx_preamble(zo_c16* out640);                                /* createPreamble.blk */
void zo_tx_symbol(const zo_c16* sub48, int k, zo_c16* out160);      /* map_ofdm >>> ifft */
int  zo_tx_packet(const uint8_t* in, int nin, zo_c16* out, int max_out);   /* transmitter() */

#ifdef __cplusplus
}
#endif
#endif
