/*
 * ziria_rx.h — C-ABI of the MI355X (gfx950) 802.11a RX decode engine, libziria_rx.so.
 *
 * Part 1 re-exports the reference's own external bricks with identical signatures and
 * per-call semantics.  wplc emits every `fun external f` as a prototype `__ext_f(...)` with
 * each array argument expanded to (pointer, length) (src/Codegen/CgFun.hs:287-316,
 * src/Codegen/CgCall.hs:72-130) into a test.cpp that the reference builds with g++
 * (csrc/Makefile:92-96), i.e. with C++ linkage and the reference's types (num8 = char,
 * int16 = short, int32 = int; csrc/numerics.h:64-69, csrc/types.h:32-33).  So the library
 * exports each external twice: with those C++ (mangled) names, which a C++ includer of this
 * header sees and a wplc-compiled program links against unchanged, and with C linkage
 * (unmangled), which a C includer and ctypes see.  The per-call externals run on the host
 * CPU ("a CPU path, with the GPU used only if batched").
 *
 * Part 2 adds batched counterparts over host arrays, run on the GPU.  They use only arrays
 * and scalars, so they can be declared in a .blk file as `fun external` (INTEGRATION.md
 * shows the declarations); like Part 1 they are exported with both linkages.
 *
 * Part 3 is the throughput API over device-resident buffers (HBM), asynchronous on a
 * caller-provided HIP stream; this is what bench.py and the Python engine drive.  C linkage.
 *
 * All buffers are caller-owned.  Status-returning functions return ZRX_OK (0) or a
 * negative ZRX_E* code; the reference's own externals keep their reference return values.
 */
#ifndef ZIRIA_RX_H
#define ZIRIA_RX_H
#include <stdint.h>

/* csrc/numerics.h:113-116 */
struct complex16 { int16_t re; int16_t im; };

/* Parts 1 and 2: C++ linkage for C++ includers (the names wplc output links against); C
 * linkage for C includers and inside the library's C-linkage translation units. */
#if defined(__cplusplus) && defined(ZRX_C_LINKAGE_EXTERNALS)
extern "C" {
#endif

/* ================================================================ Part 1: reference bricks */

/* Replaces __ext_sora_fft (reference csrc/sora_ext_lib.cpp:2672-2812, declared
 * lib/externals.blk:201-202): FFTSafe<nFFTSize> on the host CPU for every size the
 * reference dispatches (16, 32, ..., 2048 and the LTE sizes 12 .. 1200, listed at
 * zrx_fft_dev, the batched GPU counterpart); any other size prints the reference's error
 * message and leaves `out` untouched, as the reference does (:2808-2810).  in/out may alias. */
void __ext_sora_fft(struct complex16* out, int nFFTSize, struct complex16* in, int unused1);

/* Replaces __ext_sora_fft_dynamic (sora_ext_lib.cpp:2816-2820, externals.blk:205-206). */
void __ext_sora_fft_dynamic(struct complex16* out, int unused2, int16_t nFFTSize,
                            struct complex16* in, int unused1);

/* Replaces __ext_viterbi_brick_init_fast (csrc/sora_ext_viterbi.cpp:48-63,
 * externals.blk:215).  Resets the (single, global, non-reentrant) streaming decoder; like
 * the reference it keeps frame_len as an unsigned 16-bit value. */
int __ext_viterbi_brick_init_fast(int32_t frame_len, int16_t code_rate, int16_t depth);

/* Replaces __ext_viterbi_brick_decode_fast (sora_ext_viterbi.cpp:66-153,
 * externals.blk:216): consumes len1 soft values (whole groups of 2/3/4 for rate 1/2, 2/3,
 * 3/4), runs the brick's normalize and traceback schedule, writes the bytes this call
 * decodes to bit[0..] (LSB-first bits) and returns their bit count.  Like the reference it
 * does not bound the writes by len2.  The trellis holds 40000 columns (TRELLIS_MAX, :39):
 * groups beyond it are not consumed (the reference writes past its buffer). */
int16_t __ext_viterbi_brick_decode_fast(char* intInput, int len1, unsigned char* bit, int len2);

/* Replaces __ext_viterbiSig11a_brick_init_fast (sora_ext_viterbi.cpp:158-173). */
int __ext_viterbiSig11a_brick_init_fast(int32_t frame_len, int16_t code_rate, int16_t depth);

/* Replaces __ext_viterbiSig11a_brick_decode_fast (sora_ext_viterbi.cpp:176-194,
 * externals.blk:217): 48 soft values -> 24 PLCP bits; like the reference it then shifts
 * the 32-bit word at `bit` right by 6 (so `bit` must hold 4 bytes).  Returns 0. */
int16_t __ext_viterbiSig11a_brick_decode_fast(char* intInput, int len1, unsigned char* bit, int len2);

/* Replaces __ext_v_shift_right_complex16 (sora_ext_lib.cpp:1979-1995, externals.blk:110). */
int __ext_v_shift_right_complex16(struct complex16* z, int unused3, struct complex16* x, int len,
                                  int shift);

/* ================================================================ Part 2: batched, host arrays */

/* nsym independent 64-point FFTs: in/out hold 64*nsym complex16 (inlen = outlen = 64*nsym). */
void __ext_sora_fft64_batch(struct complex16* out, int outlen, struct complex16* in, int inlen);

/* Batched Viterbi.  Packet i decodes soft[pkt_soft_off[i] .. pkt_soft_off[i+1]) exactly as
 * init(frame_len[i], code_rate[i], 256) followed by decode calls over all its soft values,
 * writing its bytes at out_bits[pkt_out_off[i] ..] (byte offsets; bytes are LSB-first bit
 * arrays).  pkt_soft_off has npkts+1 entries; every per-packet soft count must be a multiple
 * of 48, and the frames' output ranges [pkt_out_off[i], +frame_len[i]) must not overlap
 * (ZRX_EINVAL).  Only the bytes a frame decoded are written; the rest of its range and every
 * byte between ranges keep the caller's contents.  Returns the number of packets decoded, or a
 * negative ZRX_E* code. */
int32_t __ext_viterbi_batch_decode(char* soft, int softlen, int32_t* pkt_soft_off, int n_off,
                                   int32_t* frame_len, int n_fl, int16_t* code_rate, int n_cr,
                                   unsigned char* out_bits, int out_len_bits,
                                   int32_t* pkt_out_off, int n_oo);

/* Batched receiveBits (code/WiFi/receiver/receiver.blk:43-54) behind FFT (OFDM/FFT.blk) and
 * GetData: packet i = symbols [pkt_sym_off[i], pkt_sym_off[i+1]) of `sym` (64 complex16 per
 * CP-removed OFDM symbol; the first is the SIGNAL symbol).  Writes the descrambled payload
 * (len-4 bytes) of packet i at payload[i*4096 ..] and pkt_info[8*i ..] = {modulation,
 * coding, len, header_err, crc_ok, status, symbols_used, viterbi_bits}.  Only the first len-4
 * bytes of a slot are defined: the rest may be zeros or keep the caller's bytes (this call
 * writes a slot only as far as the widest payload its packets' symbol counts allow).
 * Returns the number of packets whose CRC passed, or a negative ZRX_E* code.
 *
 * Every batched call of Part 2 is split into contiguous packet ranges over the node's GPUs
 * (zrx_set_devices: by default every visible gfx950 device), one host thread, context and
 * PCIe link per GPU, each range's outputs written straight into the caller's arrays; no data
 * moves between GPUs.  Calls are serialized (one at a time, like the reference's global
 * decoder), and the caller's current HIP device is left as it was. */
int32_t __ext_wifi_rx_batch(struct complex16* sym, int nsym_total, int32_t* pkt_sym_off, int n_off,
                            unsigned char* payload, int payload_len_bits,
                            int32_t* pkt_info, int n_info);

/* The same with ChannelEqualization and PilotTrack between FFT and GetData, i.e. the
 * receiver order FFT >>> ChannelEqualization(params) >>> PilotTrack >>> GetData >>>
 * receiveBits of code/WiFi/receiver/receiver.blk:66-71 (OFDM/ChannelEqualization.blk:26-46,
 * OFDM/PilotTrack.blk:56-249).  chan holds the 64 LTS channel coefficients
 * (LTECoeffs.channelCoeffs, const.blk:59-61) of each packet: chan[64*i .. 64*i+63],
 * chan_len >= 64*npkts. */
int32_t __ext_wifi_rx_eq_batch(struct complex16* sym, int nsym_total, int32_t* pkt_sym_off, int n_off,
                               struct complex16* chan, int chan_len, unsigned char* payload,
                               int payload_len_bits, int32_t* pkt_info, int n_info);

/* receiver() of code/WiFi/receiver/receiver.blk:57-72 once per capture: capture i =
 * samples[cap_off[i] .. cap_off[i+1]) (complex16, the receiver's input; downsample != 0
 * first applies downSample.blk, keeping the odd samples of every 8).  removeDC >>>
 * cca(1000) finds the preamble (cca/cca_tufv.blk), LTS (OFDM/LTS.blk) estimates the channel,
 * DataSymbol strips the cyclic prefix, then the decode chain runs with ChannelEqualization
 * and PilotTrack.  payload / pkt_info as __ext_wifi_rx_batch; det[8*i ..] = {detected,
 * noSamples, shift, energy, noise, maxCorr (CCAParams, const.blk:51-57), samples consumed by
 * the detection, first data sample}.  Returns the number of captures with a detected
 * packet whose CRC passed.  Only the first len-4 bytes of a
 * payload slot are defined, as for __ext_wifi_rx_batch. */
int32_t __ext_wifi_rx_stream_batch(struct complex16* samples, int nsamples, int32_t* cap_off, int n_off,
                                   int downsample, unsigned char* payload, int payload_len_bits,
                                   int32_t* pkt_info, int n_info, int32_t* det, int n_det);

/* transmitter() of code/WiFi/transmitter/transmitter.blk:128-133 per packet, at its default
 * 40 MHz oversampling (128-point IFFT, 32-sample cyclic prefix): packet i = in[pkt_in_off[i]
 * .. pkt_in_off[i+1]) = 3 PLCP header bytes (emitHeader: RATE, LENGTH, parity, tail as the
 * air bits) then LENGTH-4 payload bytes.  Writes 640 preamble samples + 160 per OFDM symbol
 * (SIGNAL + data) at out[pkt_out_off[i] ..] (n_oo >= npkts+1 offsets filled by the call).
 * Returns the total number of complex16 samples written, or a negative ZRX_E* code. */
int32_t __ext_wifi_tx_batch(unsigned char* in, int inlen, int32_t* pkt_in_off, int n_off,
                            struct complex16* out, int outlen, int32_t* pkt_out_off, int n_oo);

#if defined(__cplusplus) && defined(ZRX_C_LINKAGE_EXTERNALS)
}
#endif

/* ================================================================ Part 3: device API */
#ifdef __cplusplus
extern "C" {
#endif

#define ZRX_OK 0
#define ZRX_EINVAL (-1)    /* bad argument (sizes, rates, soft count not a group multiple) */
#define ZRX_EHIP (-2)      /* HIP runtime error */
#define ZRX_ENOMEM (-3)    /* workspace too small / allocation failed */
#define ZRX_ENODEV (-4)    /* no gfx950 device */
#define ZRX_EPLAN (-5)     /* the Viterbi plan dropped rows past its bound (zrx_plan_check) */
#define ZRX_EINTERNAL (-6) /* an internal consistency check failed (a bug: reported, never silent) */

/* packet status in pkt_info[5] */
#define ZRX_PKT_OK 0
#define ZRX_PKT_HDR_ERR 1      /* PLCP header parity/tail/length error: no payload (as the reference) */
#define ZRX_PKT_TRUNCATED 2    /* fewer symbols than the header requires */
#define ZRX_PKT_OVERSIZE 3     /* header needs more symbols than the reserved workspace holds (zrx_reserve) */

typedef struct zrx_ctx zrx_ctx;

/* Engine context on `device` issuing on `stream` (hipStream_t, may be NULL = default). */
int zrx_create(zrx_ctx** ctx, int device, void* stream);
int zrx_destroy(zrx_ctx* ctx);
int zrx_set_stream(zrx_ctx* ctx, void* stream);
/* Pre-allocates the workspace for rx batches of up to npkts packets whose largest
 * packet has max_nsym symbols (no allocation happens inside the launch functions). */
int zrx_reserve(zrx_ctx* ctx, int npkts, int max_nsym);
/* Per-stage HIP-event timing on the context's stream (0 = off).  Turning it on (or off)
 * starts a new measurement: every zrx_rx_dev launch from then on records its own events. */
int zrx_enable_timing(zrx_ctx* ctx, int on);
/* Average stage durations (ms) over the launches recorded since zrx_enable_timing or the
 * previous zrx_get_timing: [0] SIGNAL FFT+demap, [1] SIGNAL Viterbi+header, [2] data
 * FFT+demap+deinterleave, [3] data Viterbi, [4] descramble+CRC.  Synchronizes; all zero
 * if nothing was recorded. */
int zrx_get_timing(zrx_ctx* ctx, float* ms5);

/* Two contexts taking a stream of rx batches in turn (two batches in flight, each on its own
 * stream).  mode 0 unlinks them; with bit 0 set a context's data Viterbi waits until the
 * peer's last launched chain has finished (so the Viterbi grid is always placed on an
 * otherwise idle GPU); with bit 1 its data FFT waits until the peer's last launched data
 * Viterbi has finished; with bit 2 its chain's head (SIGNAL, plan, data FFT) runs on a
 * lowest-priority stream of its own, forked from and joined back into the context's stream,
 * so the peer's Viterbi blocks are dispatched ahead of it; with bits 0 and 3 the data Viterbi
 * waits only for the peer's last data Viterbi and seam pass (the peer's descramble/CRC then
 * overlaps it).  Event waits and stream choice only: results never change. */
int zrx_pipeline_link(zrx_ctx* a, zrx_ctx* b, int mode);

/* d_in/d_out: 64*nsym complex16 each (may alias). */
int zrx_fft64_dev(zrx_ctx* ctx, const struct complex16* d_in, struct complex16* d_out, int64_t nsym);
/* FFTSafe<nfft> (csrc/fft_r4difx.hpp:220-237) of count consecutive blocks of nfft complex16
 * (d_in/d_out may alias), for every size __ext_sora_fft dispatches: 16, 32, ..., 2048 and the
 * LTE sizes 12, 24, 36, 48, 60, 72, 96, 108, 120, 144, 180, 192, 216, 240, 288, 300, 324,
 * 360, 384, 432, 480, 540, 576, 600, 648, 720, 768, 864, 900, 960, 972, 1080, 1152, 1200.
 * ZRX_EINVAL for any other size. */
int zrx_fft_dev(zrx_ctx* ctx, int nfft, const struct complex16* d_in, struct complex16* d_out, int64_t count);

/* d_params: 4 int32 per packet {frame_len, code_rate, soft_len, 0}; d_soft_off, d_out_off:
 * int64 byte offsets per packet; d_out_bits: int32 per packet (bits written, or -1 for a
 * packet of more than 4 GiB of soft values). */
int zrx_viterbi_dev(zrx_ctx* ctx, const int8_t* d_soft, const int64_t* d_soft_off,
                    const int32_t* d_params, int npkts, uint8_t* d_out, const int64_t* d_out_off,
                    int32_t* d_out_bits);

/* The Viterbi plan of the context's last zrx_viterbi_dev / zrx_rx_dev launch (synchronizes):
 * stats2[0] = decoder rows (frames, or their trellis segments when the batch was too small
 * to fill the GPU), stats2[1] = frames the seam pass re-decoded from a seam whose two
 * segments disagreed (DESIGN.md "Trellis segments"). */
int zrx_plan_stats(zrx_ctx* ctx, int32_t* stats2);
/* ZRX_OK, or ZRX_EPLAN if the last plan dropped rows past the bound its workspace was sized
 * for (those packets would be left undecoded; never expected).  Synchronizes. */
int zrx_plan_check(zrx_ctx* ctx);

/* Full chain; d_sym_off: int64 symbol index of each packet's SIGNAL symbol; d_nsym: int32
 * symbols available per packet; max_nsym: the largest d_nsym, which must fit the reserved
 * workspace (zrx_reserve).  The device never writes past a packet's workspace slot: a packet
 * whose PLCP header needs more symbols than the workspace holds (possible only when d_nsym
 * exceeds the reservation) gets status ZRX_PKT_OVERSIZE and no payload.  d_payload holds
 * npkts*4096 bytes, d_info npkts*8 int32 (layout as __ext_wifi_rx_batch). */
int zrx_rx_dev(zrx_ctx* ctx, const struct complex16* d_sym, const int64_t* d_sym_off,
               const int32_t* d_nsym, int npkts, int max_nsym, uint8_t* d_payload,
               int32_t* d_info);

/* Full chain with ChannelEqualization + PilotTrack (as __ext_wifi_rx_eq_batch); d_chan: 64
 * complex16 channel coefficients per packet. */
int zrx_rx_eq_dev(zrx_ctx* ctx, const struct complex16* d_sym, const int64_t* d_sym_off,
                  const int32_t* d_nsym, int npkts, int max_nsym, const struct complex16* d_chan,
                  uint8_t* d_payload, int32_t* d_info);

/* FFT >>> ChannelEqualization >>> PilotTrack over every symbol of every packet (symbol k of
 * packet i is d_sym[64*(d_sym_off[i]+k) ..], k < d_nsym[i]; k = 0 is the SIGNAL symbol,
 * which PilotTrack counts as its first).  d_out has d_sym's layout and receives
 * PilotTrack's 64-bin output. */
int zrx_ofdm_eq_dev(zrx_ctx* ctx, const struct complex16* d_sym, const int64_t* d_sym_off,
                    const int32_t* d_nsym, int npkts, const struct complex16* d_chan,
                    struct complex16* d_out);

/* receiver() per capture on device buffers (as __ext_wifi_rx_stream_batch); d_cap_off int64,
 * d_cap_len int32 in input samples, max_len >= every d_cap_len (sizes the symbol staging,
 * which grows on first use), d_det 8 int32 per capture. */
int zrx_rx_stream_dev(zrx_ctx* ctx, const struct complex16* d_samples, const int64_t* d_cap_off,
                      const int32_t* d_cap_len, int ncap, int max_len, int downsample,
                      uint8_t* d_payload, int32_t* d_info, int32_t* d_det);

/* transmitter() per packet on device buffers (as __ext_wifi_tx_batch): d_in_off int64 byte
 * offsets, d_out_off int64 sample offsets with room for zrx_tx_samples(header) samples,
 * d_nsamp receives each packet's sample count. */
int zrx_tx_dev(zrx_ctx* ctx, const uint8_t* d_in, const int64_t* d_in_off, int npkts,
               struct complex16* d_out, const int64_t* d_out_off, int32_t* d_nsamp);
/* Samples transmitter() emits for a packet with these 3 PLCP header bytes (host, no GPU). */
int zrx_tx_samples(const uint8_t* hdr3);
/* Host-side copy of the 640-sample 40 MHz preamble (createPreamble.blk). */
int zrx_tx_preamble(int16_t* out1280);

/* Host-side copy of the STS correlation pattern of cca (cca_tufv.blk:80-98), 16 x 16
 * complex16.  No GPU needed. */
int zrx_cca_pattern(int16_t* pattern512);

/* Host-side copy of the engine's integer trig tables (sinx, cosx: 65536 entries by
 * unsigned angle; atan2x: 256x256 by (u8)y, (u8)x), csrc/intalglutx.h.  No GPU needed. */
int zrx_trig_tables(int16_t* sin65536, int16_t* cos65536, int16_t* atan65536);

/* ---- The node behind the batched externals of Part 2 (no device buffers involved). */

/* The logical shards a batched call is split over: n device ids (a device may repeat, giving
 * it several shards, each with its own context, stream and host thread), or n = 0 for the
 * default: the ZRX_DEVICES environment list ("0,1,2,3"), else every visible gfx950 device.
 * A call is split into at most min(shards, max(1, input bytes / min_shard_bytes)) contiguous
 * packet ranges of nearly equal input bytes (min_shard_bytes < 0: the default, 16 MiB; 0:
 * always every shard).  Drops the previous shard contexts.  ZRX_ENODEV if a listed device is
 * not a gfx950 device. */
int zrx_set_devices(const int32_t* devices, int n, int64_t min_shard_bytes);
/* The shard list in use (resolving the default): writes up to cap device ids and returns the
 * number of shards, or a negative ZRX_E* code (ZRX_ENODEV without a gfx950 device). */
int zrx_get_devices(int32_t* devices, int cap);
/* stats8 = {shards the last batched call ran on, host-register mode, caller ranges the library
 * holds page-locked, their bytes, registrations made, calls that found their arrays already
 * registered, registrations that failed, min_shard_bytes}. */
int zrx_node_stats(int64_t* stats8);
/* Page-locking of the caller's host arrays, so their copies skip the pinned staging slots:
 * 0 = never; 1 (default, or ZRX_HOST_REGISTER=1) = arrays in the main program's static
 * storage (.data/.bss: where wplc puts a program's arrays; never unmapped), registered on first
 * use and kept; 2 = also any other array of at least 32 KiB, on first use -- the caller keeps
 * those arrays mapped until it sets mode 0 or 1, which releases them (a page-lock must not
 * outlive its memory).  Memory the caller pinned itself is always used in place. */
int zrx_set_host_register(int mode);
/* The split rule of zrx_set_devices on its own (host only, no GPU): packet i weighs
 * prefix[i+1] - prefix[i] (np+1 non-decreasing entries); writes cut[0..k] (room for
 * nshards+1) and returns k, the number of ranges [cut[j], cut[j+1]). */
int zrx_shard_split(const int64_t* prefix, int np, int nshards, int64_t min_bytes, int32_t* cut);
/* Host-only check of the shard runner (no GPU): splits as zrx_shard_split, runs one thread per
 * range writing owner[i] = range index for its packets and merges their counts as a batched
 * call does; the range fail_shard (or none, -1) returns ZRX_EINTERNAL instead.  Returns np,
 * or the first failing range's code. */
int zrx_shard_selftest(const int64_t* prefix, int np, int nshards, int64_t min_bytes, int32_t* owner,
                       int fail_shard);

/* Version / build string. */
const char* zrx_version(void);

#ifdef __cplusplus
}
#endif
#endif
