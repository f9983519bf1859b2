/*
 * ORACLE — test infrastructure only (see ziria_oracle.h).
 *
 * ChannelEqualization + PilotTrack, the first "next" row of SURVEY.md §8f, restated from
 * code/WiFi/receiver/OFDM/ChannelEqualization.blk:26-46 and OFDM/PilotTrack.blk:56-249 with
 * the integer trigonometry of csrc/intalgx.h:38-99 and __ext_v_mul_complex16
 * (csrc/sora_ext_lib.cpp:2098-2137).  Pinned against the reference's KATs
 * code/WiFi/receiver/tests/test_c_{ChannelEqualization,PilotTrack}.* and, for the trig
 * tables and v_mul, against the reference bricks compiled from /root/reference
 * (oracle/ref_harness_fft.cpp).
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "ziria_oracle.h"

/* ---- integer trigonometry ------------------------------------------------------------
 * sinx / cosx index a 65536-entry table by (unsigned short) angle, FP_RAD pi = 0x8000
 * (intalgx.h:38-46); atan2x (:88-99) scales (y, x) by a common right shift until both
 * fit a signed byte and reads atan2x_lut[(u8)y][(u8)x].  The tables
 * (csrc/intalglutx.h:23, :3667, :7351) are regenerated from their closed forms, which use
 * pi written as 3.141593:
 *   sinx_lut[r] = rint(32767 sin(2 r 3.141593 / 65536)), cosx_lut likewise with cos;
 *   atan2x_lut[(u8)y][(u8)x] = trunc(atan2(y, x) / 3.141593 * 32768).
 * tests/test_oracle_vs_ref.py compares every entry with the reference tables. */
#define ZO_PI_LUT 3.141593
static int16_t g_sin[65536], g_cos[65536], g_atan[65536];
static int g_psgn[128];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

int16_t zo_trig_sin_entry(int r) { return (int16_t)nearbyint(32767.0 * sin((double)(r & 0xFFFF) * 2.0 * ZO_PI_LUT / 65536.0)); }
int16_t zo_trig_cos_entry(int r) { return (int16_t)nearbyint(32767.0 * cos((double)(r & 0xFFFF) * 2.0 * ZO_PI_LUT / 65536.0)); }
int16_t zo_trig_atan2_entry(int yy, int xx) {     /* yy, xx in [-128, 127] */
  return (int16_t)trunc(atan2((double)yy, (double)xx) / ZO_PI_LUT * 32768.0);
}
static void tables_init(void) {
  for (int r = 0; r < 65536; r++) {
    g_sin[r] = zo_trig_sin_entry(r);
    g_cos[r] = zo_trig_cos_entry(r);
  }
  for (int i = 0; i < 256; i++)
    for (int j = 0; j < 256; j++) g_atan[(i << 8) | j] = zo_trig_atan2_entry((int8_t)i, (int8_t)j);
  /* pilotSgn (PilotTrack.blk:70-78): entry m = polarity p_{(m+1) mod 127} of the 802.11a
     pilot sequence (0 = +1, -1 = -1), the scrambler (scramble.blk:28-44) output from the
     all-ones state */
  int s[7] = {1, 1, 1, 1, 1, 1, 1}, p[127];
  for (int k = 0; k < 127; k++) {
    const int t = s[3] ^ s[0];
    for (int j = 0; j < 6; j++) s[j] = s[j + 1];
    s[6] = t;
    p[k] = t;
  }
  for (int m = 0; m < 128; m++) g_psgn[m] = p[(m + 1) % 127] ? -1 : 0;
  /* both reference tables (this one and allPilotSgn, transmitter/map_ofdm.blk:30-38) hold
     +1 at entry 52 where the 802.11a sequence has p_53 = -1; kept as in the reference */
  g_psgn[52] = 0;
}
int16_t zo_sin16(int16_t r) { pthread_once(&g_once, tables_init); return g_sin[(uint16_t)r]; }
int16_t zo_cos16(int16_t r) { pthread_once(&g_once, tables_init); return g_cos[(uint16_t)r]; }
int zo_pilot_sign(int m) { pthread_once(&g_once, tables_init); return g_psgn[m & 127]; }

/* bit_scope_s (intalgx.h:50-85): index of the highest set bit of |x| (0 for x = 0) */
static int bit_scope(int x) {
  const unsigned u = x > 0 ? (unsigned)x : (unsigned)(-x);
  return u ? 31 - __builtin_clz(u) : 0;
}
int16_t zo_atan2_16(int16_t y, int16_t x) {
  pthread_once(&g_once, tables_init);
  const int ys = bit_scope(y), xs = bit_scope(x);
  const int shift = (xs > ys ? xs : ys) - 6;
  int yy = y, xx = x;
  if (shift > 0) { yy = y >> shift; xx = x >> shift; }
  return g_atan[((unsigned)(uint8_t)yy << 8) | (uint8_t)xx];
}

/* ---- __ext_v_mul_complex16 (sora_ext_lib.cpp:2098-2137) ------------------------------
 * Groups of 4: im negated in 16 bits (xor 0xFFFF0000, + 0x10000), _mm_madd_epi16 (two
 * exact products, 32-bit wrapping sum), arithmetic shift, low 16 bits.  The scalar tail
 * (len % 4) computes in int. */
void zo_v_mul_complex16(zo_c16* out, const zo_c16* x, const zo_c16* y, int len, int shift) {
  const int full = len / 4 * 4;
  for (int i = 0; i < full; i++) {
    const int16_t nim = (int16_t)(uint16_t)(-(int32_t)x[i].im);
    const uint32_t re = (uint32_t)((int32_t)x[i].re * y[i].re) + (uint32_t)((int32_t)nim * y[i].im);
    const uint32_t im = (uint32_t)((int32_t)x[i].im * y[i].re) + (uint32_t)((int32_t)x[i].re * y[i].im);
    out[i].re = (int16_t)((int32_t)re >> shift);
    out[i].im = (int16_t)((int32_t)im >> shift);
  }
  for (int i = full; i < len; i++) {
    const int32_t re = (int32_t)((uint32_t)((int32_t)x[i].re * y[i].re) - (uint32_t)((int32_t)x[i].im * y[i].im));
    const int32_t im = (int32_t)((uint32_t)((int32_t)x[i].re * y[i].im) + (uint32_t)((int32_t)x[i].im * y[i].re));
    out[i].re = (int16_t)(re >> shift);
    out[i].im = (int16_t)(im >> shift);
  }
}

/* ---- ChannelEqualization.blk:26-46 (norm_shift = 8, const.blk:27) ------------------- */
void zo_channel_eq(const zo_c16* in, const zo_c16* co, zo_c16* out) {
  zo_c16 t[64];
  memcpy(t + 28, in + 28, 8 * sizeof(zo_c16));
  zo_v_mul_complex16(t, in, co, 28, 8);
  zo_v_mul_complex16(t + 36, in + 36, co + 36, 28, 8);
  memcpy(out, t, sizeof(t));
}

/* ---- PilotTrack.blk:56-249 -----------------------------------------------------------
 * k: index of the symbol in the packet (0 = SIGNAL): symbol_count starts at 127 and wraps
 * to 0 after each symbol (:58, :180-183).  The CFO/SFO trackers and the pilot history
 * (:152-170, :209-215) do not reach the output (CFO compensation is disabled, :107-111,
 * and `if (true)` selects the current pilots, :156), so each symbol is independent. */
void zo_pilot_track(const zo_c16* s, int k, zo_c16* out) {
  const int sc = k == 0 ? 127 : (k - 1) % 127;
  const int neg = zo_pilot_sign(sc) == -1;
  static const int pos[4] = {64 - 21, 64 - 7, 7, 21};   /* :120 */
  zo_c16 p[4];
  for (int i = 0; i < 4; i++) {
    p[i] = s[pos[i]];
    if (neg) { p[i].re = (int16_t)-p[i].re; p[i].im = (int16_t)-p[i].im; }
  }
  int32_t th[4];
  th[0] = zo_atan2_16(p[0].im, p[0].re);
  th[1] = zo_atan2_16(p[1].im, p[1].re);
  th[2] = zo_atan2_16(p[2].im, p[2].re);
  th[3] = zo_atan2_16((int16_t)-p[3].im, (int16_t)-p[3].re);
  for (int i = 0; i < 3; i++) {                      /* for i in [0,3]: unwrap (:186-196) */
    if (th[i] - th[i + 1] > 32768) th[i + 1] += 2 * 32768;
    else if (th[i + 1] - th[i] > 32768) th[i + 1] -= 2 * 32768;
  }
  const int32_t avg32 = (th[0] + th[1] + th[2] + th[3]) / 4;
  const int16_t avg = avg32 >= 32768 ? (int16_t)(avg32 - 2 * 32768)
                    : avg32 <= -32768 ? (int16_t)(avg32 + 2 * 32768) : (int16_t)avg32;
  const int16_t del = (int16_t)(((th[2] - th[0]) / (64 - pos[0] + pos[2]) +
                                 (th[3] - th[1]) / (pos[3] + 64 - pos[1])) >> 1);
  /* build_coeff (:28-50): bins 38..63, then 1..26, the angle stepping by del, dc skipped;
     bins 0 and 27..37 keep their initial zero */
  zo_c16 rot[64];
  memset(rot, 0, sizeof(rot));
  int16_t t = (int16_t)(avg - del * 26);
  for (int i = 64 - 26; i < 64; i++) {
    rot[i].re = zo_cos16(t); rot[i].im = (int16_t)-zo_sin16(t);
    t = (int16_t)(t + del);
  }
  t = (int16_t)(t + del);
  for (int i = 1; i < 27; i++) {
    rot[i].re = zo_cos16(t); rot[i].im = (int16_t)-zo_sin16(t);
    t = (int16_t)(t + del);
  }
  zo_c16 o[64];
  memset(o, 0, sizeof(o));
  zo_v_mul_complex16(o, s, rot, 28, 15);
  zo_v_mul_complex16(o + 36, s + 36, rot + 36, 28, 15);
  memcpy(out, o, sizeof(o));
}

/* FFT() >>> ChannelEqualization(params) >>> PilotTrack() (receiver.blk:66-69) */
void zo_ofdm_eq_symbol(const zo_c16* sym64, const zo_c16* chan64, int k, zo_c16* out64) {
  zo_c16 f[64], e[64];
  zo_fft64(sym64, f);
  zo_channel_eq(f, chan64, e);
  zo_pilot_track(e, k, out64);
}

/* receiver.blk:66-71 for one packet: FFT >>> ChannelEqualization >>> PilotTrack >>>
   GetData >>> receiveBits, with the packet's LTS channel coefficients chan64. */
int zo_rx_packet_time_eq(const zo_c16* sym, int nsym, const zo_c16* chan64, uint8_t* payload, zo_rx_result* r) {
  zo_c16* sub = (zo_c16*)malloc(sizeof(zo_c16) * 48 * (size_t)(nsym > 0 ? nsym : 1));
  zo_c16 e[64];
  for (int k = 0; k < nsym; k++) {
    zo_ofdm_eq_symbol(sym + 64 * k, chan64, k, e);
    zo_get_data(e, sub + 48 * k);
  }
  const int ret = zo_rx_packet_freq(sub, nsym, payload, r);
  free(sub);
  return ret;
}

typedef struct {
  int t, nt, npkts, stride;
  const zo_c16 *sym, *chan;
  const int64_t* off;
  const int32_t* nsym;
  uint8_t* payload;
  zo_rx_result* res;
} eq_job;
static void* eq_worker(void* p) {
  eq_job* j = (eq_job*)p;
  for (int i = j->t; i < j->npkts; i += j->nt)
    zo_rx_packet_time_eq(j->sym + 64 * j->off[i], j->nsym[i], j->chan + 64 * (size_t)i,
                         j->payload + (size_t)i * j->stride, &j->res[i]);
  return 0;
}
int zo_rx_batch_time_eq(const zo_c16* sym, const int64_t* sym_off, const int32_t* nsym, int npkts,
                        const zo_c16* chan, uint8_t* payload, int payload_stride, zo_rx_result* res,
                        int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  eq_job jobs[256];
  for (int t = 0; t < nthreads; t++) {
    eq_job j = {t, nthreads, npkts, payload_stride, sym, chan, sym_off, nsym, payload, res};
    jobs[t] = j;
  }
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], 0, eq_worker, &jobs[t]);
  eq_worker(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], 0);
  return 0;
}
