/*
 * ORACLE — test infrastructure only (see ziria_oracle.h).
 *
 * RX front end, the second "next" row of SURVEY.md §8f: receiver() of
 * code/WiFi/receiver/receiver.blk:57-72 over a sample stream —
 *   downSample (downSample.blk:31-57; permutatew1313 / interleave_loww,
 *     csrc/sora_ext_lib.cpp:2226-2252: keeps the odd samples),
 *   removeDC (removeDC.blk:25-85) >>> cca (cca/cca_tufv.blk:103-338, Tufvesson preamble
 *     detection with the STS pattern of :50-95, built with IFFT<64>, csrc/ifft_r4difx.hpp),
 *   LTS (OFDM/LTS.blk:29-203: AGC shift, two FFTs, calcCoeff),
 *   DataSymbol (OFDM/DataSymbol.blk:24-30: cyclic prefix removal),
 * then FFT >>> ChannelEqualization >>> PilotTrack >>> GetData >>> receiveBits
 * (ziria_oracle_eq.c, ziria_oracle.c).  Pinned by the reference's end-to-end KATs
 * code/WiFi/tests/test_rx.* and test_real_rx.*, and the IFFT against the compiled
 * reference brick.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "ziria_oracle.h"

static inline int16_t sat16(int32_t x) { return (int16_t)(x > 32767 ? 32767 : (x < -32768 ? -32768 : x)); }
static inline int16_t inv16(int16_t x) { return (int16_t)~x; }
static inline zo_c16 cadd(zo_c16 a, zo_c16 b) { zo_c16 r = {sat16(a.re + b.re), sat16(a.im + b.im)}; return r; }
static inline zo_c16 csub(zo_c16 a, zo_c16 b) { zo_c16 r = {sat16(a.re - b.re), sat16(a.im - b.im)}; return r; }
static inline zo_c16 cshr2(zo_c16 a) { zo_c16 r = {(int16_t)(a.re >> 2), (int16_t)(a.im >> 2)}; return r; }
static inline int32_t wrap32(int64_t v) { return (int32_t)(uint32_t)(uint64_t)v; }

/* ---- IFFT<64> (csrc/ifft_r4difx.hpp:56-250) ----------------------------------------- */
/* conj_mul_shiftx(a, b, 15) (csrc/sora_ext_lib_fft.hpp:68-94): a * conj(b) with the
   imaginary part's a.re complemented (XOR), madd_epi16 32-bit wrap, >> 15, low 16 bits */
static inline zo_c16 conj_mul_shift(zo_c16 a, int16_t bre, int16_t bim) {
  const int32_t re = wrap32((int64_t)a.re * bre + (int64_t)a.im * bim);
  const int32_t im = wrap32((int64_t)a.im * bre + (int64_t)inv16(a.re) * bim);
  zo_c16 r = {(int16_t)(re >> 15), (int16_t)(im >> 15)};
  return r;
}
static inline zo_c16 mul_j(zo_c16 a) { zo_c16 r = {inv16(a.im), a.re}; return r; }
/* IFFTSSE<N> (:56-97) */
static void ifft_stage(zo_c16* x, int N) {
  for (int n = 0; n < N / 4; n++) {
    zo_c16 a = cshr2(x[n]), b = cshr2(x[n + N / 4]), c = cshr2(x[n + N / 2]), d = cshr2(x[n + 3 * N / 4]);
    zo_c16 ac = cadd(a, c), bd = cadd(b, d), a_c = csub(a, c), b_d = csub(b, d);
    int16_t tr, ti;
    x[n] = cadd(ac, bd);
    zo_twiddle(N, 2, n, &tr, &ti);
    x[n + N / 4] = conj_mul_shift(csub(ac, bd), tr, ti);
    zo_c16 jb = mul_j(b_d);
    zo_twiddle(N, 1, n, &tr, &ti);
    x[n + N / 2] = conj_mul_shift(cadd(a_c, jb), tr, ti);
    zo_twiddle(N, 3, n, &tr, &ti);
    x[n + 3 * N / 4] = conj_mul_shift(csub(a_c, jb), tr, ti);
  }
}
/* IFFTSSEEx<4> (:114-150): with y = x >> 2, A = y0+y2, B = y1+y3, C = y0+~y2, D = y1+~y3
   (saturating), jD = (~D.im, D.re): outputs A+B, A+~B, C+jD, C+~jD. */
static void ifft4(zo_c16* x) {
  const zo_c16 y0 = cshr2(x[0]), y1 = cshr2(x[1]), y2 = cshr2(x[2]), y3 = cshr2(x[3]);
  const zo_c16 A = cadd(y0, y2), B = cadd(y1, y3);
  const zo_c16 ny2 = {inv16(y2.re), inv16(y2.im)}, ny3 = {inv16(y3.re), inv16(y3.im)};
  const zo_c16 C = cadd(y0, ny2), D = cadd(y1, ny3);
  const zo_c16 jD = {inv16(D.im), D.re};
  const zo_c16 nB = {inv16(B.re), inv16(B.im)}, njD = {inv16(jD.re), inv16(jD.im)};
  x[0] = cadd(A, B);
  x[1] = cadd(nB, A);
  x[2] = cadd(C, jD);
  x[3] = cadd(njD, C);
}
static int bitrev6(int i) {
  int r = 0;
  for (int b = 0; b < 6; b++) r |= ((i >> b) & 1) << (5 - b);
  return r;
}
/* IFFT<64> / IFFTSafe<64> (:231-248): output through the 6-bit bit reversal */
void zo_ifft64(const zo_c16* in, zo_c16* out) {
  zo_c16 x[64];
  memcpy(x, in, sizeof(x));
  ifft_stage(x, 64);
  for (int q = 0; q < 4; q++) {
    ifft_stage(x + 16 * q, 16);
    for (int r = 0; r < 4; r++) ifft4(x + 16 * q + 4 * r);
  }
  for (int i = 0; i < 64; i++) out[i] = x[bitrev6(i)];
}

/* ---- small vector externals ----------------------------------------------------------- */
/* __ext_v_conj_mul_complex16_int32 (sora_ext_lib.cpp:2144-2174): x * conj(y) in int32:
   re = y.re x.re + y.im x.im, im = x.im y.re - x.re y.im (16-bit negated y.im, madd wrap) */
static void conj_mul_i32(const zo_c16* x, const zo_c16* y, int n, int32_t* re, int32_t* im) {
  for (int i = 0; i < n; i++) {
    const int16_t nyim = (int16_t)(uint16_t)(-(int32_t)y[i].im);
    re[i] = wrap32((int64_t)y[i].re * x[i].re + (int64_t)y[i].im * x[i].im);
    im[i] = wrap32((int64_t)nyim * x[i].re + (int64_t)y[i].re * x[i].im);
  }
}
/* __ext_v_shift_left_complex16 (:1998-2015): _mm_slli_epi16 (logical, wrapping) */
static void shl_c16(zo_c16* z, const zo_c16* x, int n, int sh) {
  for (int i = 0; i < n; i++) {
    z[i].re = (int16_t)(sh > 15 ? 0 : (uint16_t)((uint16_t)x[i].re << sh));
    z[i].im = (int16_t)(sh > 15 ? 0 : (uint16_t)((uint16_t)x[i].im << sh));
  }
}

/* ---- downSample (downSample.blk:31-57) ------------------------------------------------ */
int zo_downsample(const zo_c16* in, int n, zo_c16* out) {
  const int groups = n / 8;                       /* takes 8, emits 4 */
  for (int g = 0; g < groups; g++)
    for (int k = 0; k < 4; k++) out[4 * g + k] = in[8 * g + 2 * k + 1];
  return 4 * groups;
}

/* ---- removeDC (removeDC.blk:25-85), 4 samples per step -------------------------------- */
typedef struct { zo_c16 sum_dc[4], dc[4]; int cnt; } dc_state;
static void dc_init(dc_state* s) { memset(s, 0, sizeof(*s)); s->cnt = 8; }
static void dc_step(dc_state* s, const zo_c16* x, zo_c16* y) {
  for (int k = 0; k < 4; k++) {                  /* v_sub_complex16: wrapping 16-bit */
    y[k].re = (int16_t)(x[k].re - s->dc[k].re);
    y[k].im = (int16_t)(x[k].im - s->dc[k].im);
  }
  zo_c16 tmp[4];
  zo_v_shift_right_complex16(tmp, y, 4, 5);
  /* v_hadd_complex16 (sora_ext_lib.cpp:1847-1858): num16 sums, broadcast */
  const int16_t hr = (int16_t)(tmp[0].re + tmp[1].re + tmp[2].re + tmp[3].re);
  const int16_t hi = (int16_t)(tmp[0].im + tmp[1].im + tmp[2].im + tmp[3].im);
  for (int k = 0; k < 4; k++) {                  /* v_add_complex16: wrapping */
    s->sum_dc[k].re = (int16_t)(hr + s->sum_dc[k].re);
    s->sum_dc[k].im = (int16_t)(hi + s->sum_dc[k].im);
  }
  if (s->cnt == 0) {
    zo_v_shift_right_complex16(tmp, s->sum_dc, 4, 2);
    for (int k = 0; k < 4; k++) {
      s->dc[k].re = (int16_t)(tmp[k].re + s->dc[k].re);
      s->dc[k].im = (int16_t)(tmp[k].im + s->dc[k].im);
    }
    s->cnt = 8;
    memset(s->sum_dc, 0, sizeof(s->sum_dc));
  }
  s->cnt--;
}

/* removeDC over a stream (whole 4-sample steps) */
int zo_remove_dc(const zo_c16* x, int n, zo_c16* y) {
  dc_state s;
  dc_init(&s);
  const int steps = n / 4;
  for (int i = 0; i < steps; i++) dc_step(&s, x + 4 * i, y + 4 * i);
  return 4 * steps;
}

/* ---- cca (cca/cca_tufv.blk) ------------------------------------------------------------ */
#define CORR_LEN 16
#define NO_REP 9
/* createSTSinTime (:50-77) + InitCorrPattern (:80-98): pattern[16 i + j] = sts_time[i + j] >> 7 */
void zo_cca_pattern(zo_c16* pattern) {
  const int16_t m = (int16_t)(10720.0 * 1.472);   /* bpsk_mod_11a (const.blk:29) * 1.472 */
  zo_c16 sts[64], t[64];
  memset(sts, 0, sizeof(sts));
  const int pos[12] = {4, 8, 12, 16, 20, 24, 40, 44, 48, 52, 56, 60};
  const int sgn[12] = {-1, -1, 1, 1, 1, 1, 1, -1, 1, -1, -1, 1};
  for (int i = 0; i < 12; i++) { sts[pos[i]].re = (int16_t)(sgn[i] * m); sts[pos[i]].im = (int16_t)(sgn[i] * m); }
  zo_ifft64(sts, t);
  zo_c16 pre[64];
  zo_v_shift_right_complex16(pre, t, 64, 7);
  for (int i = 0; i < CORR_LEN; i++)
    for (int j = 0; j < CORR_LEN; j++) pattern[i * CORR_LEN + j] = pre[i + j];
}
/* calcEnergy (:137-149): sum over the block of |x >> 4|^2 (two >> 2 shifts), int32 */
static int32_t calc_energy(const zo_c16* x) {
  zo_c16 a[16], b[16];
  zo_v_shift_right_complex16(a, x, 16, 2);
  zo_v_shift_right_complex16(b, a, 16, 2);
  int32_t re[16], im[16];
  conj_mul_i32(b, b, 16, re, im);
  uint32_t s = 0;
  for (int i = 0; i < 16; i++) s += (uint32_t)re[i];
  return (int32_t)s;
}
/* v_correlate (lib/v_correlate.blk:22-44): sum a1 * conj(a2) over 16 samples, int32 */
static void correlate16(const zo_c16* a1, const zo_c16* a2, int32_t* cre, int32_t* cim) {
  int32_t re[16], im[16];
  conj_mul_i32(a1, a2, 16, re, im);
  uint32_t sr[4] = {0, 0, 0, 0}, si[4] = {0, 0, 0, 0};
  for (int i = 0; i < 16; i++) { sr[i & 3] += (uint32_t)re[i]; si[i & 3] += (uint32_t)im[i]; }
  *cre = (int32_t)(sr[0] + sr[1] + sr[2] + sr[3]);
  *cim = (int32_t)(si[0] + si[1] + si[2] + si[3]);
}

/* detectPreamble = removeDC >>> cca(threshold) over stream x[0..n).  Returns 0 and fills
   det when a packet is detected; consumed = samples read (a multiple of 16). */
int zo_detect_preamble(const zo_c16* x, int n, int32_t energy_threshold, zo_cca* det, int* consumed) {
  zo_c16 pattern[CORR_LEN * CORR_LEN];
  zo_cca_pattern(pattern);
  dc_state dc;
  dc_init(&dc);
  int32_t mul_re[CORR_LEN], mul_im[CORR_LEN], corr_hist[NO_REP * CORR_LEN];
  memset(mul_re, 0, sizeof(mul_re)); memset(mul_im, 0, sizeof(mul_im));
  memset(corr_hist, 0, sizeof(corr_hist));
  int32_t oldOldCorr = 0, oldCorr = 0, maxCorr = 0, iEnergy = 0, iNoise = 0;
  int oldInd = 0, oldOldInd = 0, noInc = 0, maxInd = 0, idle_cnt = 0, iterind = 0;
  int pos = 0, idle = 0, detected = 0;
  zo_c16 blk[16];
  while (!detected) {
    if (pos + 16 > n) { *consumed = pos; return -1; }
    for (int q = 0; q < 4; q++) dc_step(&dc, x + pos + 4 * q, blk + 4 * q);
    pos += 16;
    if (!idle) {                                 /* until initial_idle (:160-179) */
      iEnergy = calc_energy(blk);
      if (iEnergy < energy_threshold) idle_cnt++; else idle_cnt = 0;
      if (idle_cnt >= 20) { idle = 1; iNoise = iEnergy; iterind = 0; }
      iterind++;
      continue;
    }
    zo_c16 input[16];                            /* until detected (:184-246) */
    zo_v_shift_right_complex16(input, blk, 16, 7);
    iEnergy = calc_energy(blk);
    maxCorr = 0;
    for (int i = 0; i < CORR_LEN; i++) {
      int32_t cre, cim;
      correlate16(pattern + i * CORR_LEN, input, &cre, &cim);
      /* corrc * conj_complex32(mul_hist[i]) (complex32_mult, csrc/numerics.c:107-113) */
      const int32_t hre = mul_re[i], him = (int32_t)(0u - (uint32_t)mul_im[i]);
      const int32_t mre = (int32_t)((uint32_t)cre * (uint32_t)hre - (uint32_t)cim * (uint32_t)him);
      const int32_t mim = (int32_t)((uint32_t)cim * (uint32_t)hre + (uint32_t)cre * (uint32_t)him);
      const int32_t corri = (int32_t)((uint32_t)(mre >= 0 ? mre : -(uint32_t)mre) +
                                      (uint32_t)(mim >= 0 ? mim : -(uint32_t)mim));
      mul_re[i] = cre; mul_im[i] = cim;
      memmove(corr_hist + i * NO_REP, corr_hist + i * NO_REP + 1, (NO_REP - 1) * sizeof(int32_t));
      corr_hist[i * NO_REP + NO_REP - 1] = corri;
      uint32_t corr = 0;
      for (int j = 0; j < NO_REP; j++) corr += (uint32_t)corr_hist[i * NO_REP + j];
      if ((int32_t)corr > maxCorr) { maxCorr = (int32_t)corr; maxInd = i; }
    }
    const int32_t norm = iEnergy == 0 ? 0 : maxCorr / iEnergy;
    if (iEnergy > energy_threshold && noInc > 4 && (oldCorr > maxCorr || oldInd != maxInd) && norm > 96)
      detected = 1;
    if (oldOldCorr < oldCorr && oldCorr < maxCorr && oldOldInd == oldInd && oldInd == maxInd) noInc++;
    else noInc = 0;
    oldOldCorr = oldCorr; oldCorr = maxCorr;
    oldOldInd = oldInd; oldInd = maxInd;
    iterind++;
  }
  det->noSamples = 16 * iterind + oldInd;        /* :331-337 */
  det->shift = oldInd;
  det->energy = iEnergy;
  det->noise = iNoise;
  det->maxCorr = maxCorr;
  *consumed = pos;
  return 0;
}

/* ---- LTS (OFDM/LTS.blk:29-203), the non-SORA_COMPAT branch ---------------------------- */
static const uint8_t LTS11A[64] = {0, 1, 0, 0, 1, 1, 0, 1, 0, 1, 0, 0, 0, 0, 0, 1,
                                   1, 0, 0, 1, 0, 1, 0, 1, 1, 1, 1, 0, 0, 0, 0, 0,
                                   0, 0, 0, 0, 0, 0, 1, 1, 0, 0, 1, 1, 0, 1, 0, 1,
                                   1, 1, 1, 1, 1, 0, 0, 1, 1, 0, 1, 0, 1, 1, 1, 1};   /* :45-49 */
/* calcCoeff (:71-111) */
static void calc_coeff(const zo_c16* f, zo_c16* ret) {
  zo_c16 lts[64];
  for (int i = 0; i < 64; i++) { lts[i].re = (int16_t)((2 * LTS11A[i] - 1) * 1600); lts[i].im = 0; }
  int32_t re[28], im[28], sq[64];
  memset(sq, 0, sizeof(sq));
  conj_mul_i32(f, f, 28, re, im);
  for (int i = 0; i < 28; i++) sq[i] = re[i] >> 6;
  conj_mul_i32(f + 36, f + 36, 28, re, im);
  for (int i = 0; i < 28; i++) sq[36 + i] = re[i] >> 6;
  conj_mul_i32(lts, f, 28, re, im);
  for (int i = 0; i < 28; i++) {
    if (sq[i] > 1) { ret[i].re = (int16_t)(re[i] / sq[i]); ret[i].im = (int16_t)(im[i] / sq[i]); }
    else { ret[i].re = 0; ret[i].im = 0; }
  }
  for (int i = 28; i < 36; i++) { ret[i].re = 0; ret[i].im = 0; }
  conj_mul_i32(lts + 36, f + 36, 28, re, im);
  for (int i = 36; i < 64; i++) {
    if (sq[i] > 1) { ret[i].re = (int16_t)(re[i - 36] / sq[i]); ret[i].im = (int16_t)(im[i - 36] / sq[i]); }
    else { ret[i].re = 0; ret[i].im = 0; }
  }
}
/* round_int32 / log2 of csrc/ext_math.c:70-80 */
static int32_t round_i32(double d) { return (int32_t)((d > 0) ? (d + 0.5) : (d - 0.5)); }
int zo_lts_agc_shift(int32_t amp) { return round_i32((log(1000.0 / sqrt((double)amp)) / log(2.0))); }
/* xp: the 144 samples LTS takes; writes the 64 channel coefficients.  compat selects the
   SORA_COMPAT branch (:189-199: calcCoeff of the first LTS only, no AGC), which is what
   receiver/tests/test_c_LTS.outfile.ground holds; the default build (no SORA_COMPAT in any
   build script) averages both LTS symbols with the AGC shift (:123-188). */
void zo_lts_coeffs_mode(const zo_c16* xp, int shift, int32_t amp, zo_c16* coeffs, int compat) {
  zo_c16 pre[64], del[64];
  memcpy(pre, xp + 16 - shift, sizeof(pre));
  memcpy(del, xp + 80 - shift, sizeof(del));
  if (compat) {
    zo_c16 f[64];
    zo_fft64(pre, f);
    calc_coeff(f, coeffs);
    return;
  }
  const int agc = zo_lts_agc_shift(amp);
  if (agc > 0) { shl_c16(pre, pre, 64, agc); shl_c16(del, del, 64, agc); }
  else { zo_v_shift_right_complex16(pre, pre, 64, -agc); zo_v_shift_right_complex16(del, del, 64, -agc); }
  zo_c16 f[64], fd[64], c1[64], c2[64];
  zo_fft64(pre, f);
  zo_fft64(del, fd);
  calc_coeff(f, c1);
  calc_coeff(fd, c2);
  for (int i = 0; i < 64; i++) {                 /* v_add_complex16: wrapping */
    coeffs[i].re = (int16_t)(c1[i].re + c2[i].re);
    coeffs[i].im = (int16_t)(c1[i].im + c2[i].im);
  }
  const int agcs = agc - 1;
  if (agcs > 0) shl_c16(coeffs, coeffs, 64, agcs);
  else zo_v_shift_right_complex16(coeffs, coeffs, 64, -agcs);
}

void zo_lts_coeffs(const zo_c16* xp, int shift, int32_t amp, zo_c16* coeffs) {
  zo_lts_coeffs_mode(xp, shift, amp, coeffs, 0);
}

/* ---- receiver() (receiver.blk:57-72) on one stream ------------------------------------- */
/* x: the receiver's input stream (after any downSample); runs detectPreamble(1000), LTS,
   DataSymbol and the decode chain.  Returns 0 on a decoded packet (r filled), <0 if no
   packet is detected or the stream ends early.  Writes the CP-removed symbols' start
   offset (in samples, relative to x) to *data_start. */
int zo_rx_stream(const zo_c16* x, int n, uint8_t* payload, zo_rx_result* r, zo_cca* det, zo_c16* coeffs,
                 int* data_start) {
  memset(r, 0, sizeof(*r));
  int used = 0;
  if (zo_detect_preamble(x, n, 1000, det, &used) != 0) return -1;
  if (used + 144 > n) return -2;
  zo_lts_coeffs(x + used, det->shift, det->maxCorr, coeffs);
  const int d0 = used + 144;
  *data_start = d0;
  const int nsym = (n - d0) / 80;
  if (nsym < 1) return -2;
  zo_c16* sym = (zo_c16*)malloc(sizeof(zo_c16) * 64 * (size_t)nsym);
  for (int k = 0; k < nsym; k++) memcpy(sym + 64 * k, x + d0 + 80 * k + 16 - det->shift, 64 * sizeof(zo_c16));
  const int ret = zo_rx_packet_time_eq(sym, nsym, coeffs, payload, r);
  free(sym);
  return ret;
}

/* ---- TX chain: transmitter() of code/WiFi/transmitter/transmitter.blk:128-133
   at the default 40 MHz oversampling (FFT_SIZE 128, CP_SIZE 32) ------------------------------ */
/* IFFTSSEEx<8> (csrc/ifft_r4difx.hpp:152-228): a = x[0..3] >> 3, b = x[4..7] >> 3; the sum
   half takes the 4-point combination of IFFTSSEEx<4> (no further shift), the difference half
   e = a - b is rotated (j e2, j e3), combined, multiplied by conj(tw8) and combined again. */
static void ifft8(zo_c16* x) {
  zo_c16 a[4], b[4], s[4], e[4];
  for (int k = 0; k < 4; k++) {
    a[k].re = (int16_t)(x[k].re >> 3); a[k].im = (int16_t)(x[k].im >> 3);
    b[k].re = (int16_t)(x[k + 4].re >> 3); b[k].im = (int16_t)(x[k + 4].im >> 3);
    s[k] = cadd(a[k], b[k]);
    e[k] = csub(a[k], b[k]);
  }
  const zo_c16 A = cadd(s[0], s[2]), B = cadd(s[1], s[3]);
  const zo_c16 C = cadd((zo_c16){inv16(s[2].re), inv16(s[2].im)}, s[0]);
  const zo_c16 D = cadd((zo_c16){inv16(s[3].re), inv16(s[3].im)}, s[1]);
  const zo_c16 jD = {inv16(D.im), D.re};
  zo_c16 o[8];
  o[0] = cadd(A, B);
  o[1] = cadd((zo_c16){inv16(B.re), inv16(B.im)}, A);
  o[2] = cadd(C, jD);
  o[3] = cadd((zo_c16){inv16(jD.re), inv16(jD.im)}, C);
  const zo_c16 je2 = {inv16(e[2].im), e[2].re}, je3 = {inv16(e[3].im), e[3].re};
  zo_c16 t[4];
  t[0] = cadd(e[0], je2);
  t[1] = cadd(e[1], je3);
  t[2] = cadd((zo_c16){inv16(je2.re), inv16(je2.im)}, e[0]);
  t[3] = cadd((zo_c16){inv16(je3.re), inv16(je3.im)}, e[1]);
  static const int16_t tw[4][2] = {{32767, 0}, {23169, -23169}, {32767, 0}, {-23169, -23169}};
  zo_c16 u[4];
  for (int k = 0; k < 4; k++) u[k] = conj_mul_shift(t[k], tw[k][0], tw[k][1]);
  o[4] = cadd(u[0], u[1]);
  o[5] = cadd((zo_c16){inv16(u[1].re), inv16(u[1].im)}, u[0]);
  o[6] = cadd(u[2], u[3]);
  o[7] = cadd((zo_c16){inv16(u[3].re), inv16(u[3].im)}, u[2]);
  memcpy(x, o, sizeof(o));
}
static int bitrev7(int i) {
  int r = 0;
  for (int b = 0; b < 7; b++) r |= ((i >> b) & 1) << (6 - b);
  return r;
}
/* IFFT<128>: IFFTSSE<128>, then per quarter IFFTSSE<32> and IFFTSSEEx<8> x 4; output
   through FFT128LUTMap (csrc/fft_lut_bitreversal.h:153), the 7-bit bit reversal */
void zo_ifft128(const zo_c16* in, zo_c16* out) {
  zo_c16 x[128];
  memcpy(x, in, sizeof(x));
  ifft_stage(x, 128);
  for (int q = 0; q < 4; q++) {
    ifft_stage(x + 32 * q, 32);
    for (int r = 0; r < 4; r++) ifft8(x + 32 * q + 8 * r);
  }
  for (int i = 0; i < 128; i++) out[i] = x[bitrev7(i)];
}

/* createSTSinTime / createLTSinTime (createPreamble.blk:38-117), 320 samples each */
void zo_tx_preamble(zo_c16* out640) {
  const int16_t sm = (int16_t)(10720.0 * 1.472), lm = 10720;
  zo_c16 f[128], t[128];
  memset(f, 0, sizeof(f));
  const int sp[12] = {4, 8, 12, 16, 20, 24, 104, 108, 112, 116, 120, 124};
  const int ss[12] = {-1, -1, 1, 1, 1, 1, 1, -1, 1, -1, -1, 1};
  for (int i = 0; i < 12; i++) { f[sp[i]].re = (int16_t)(ss[i] * sm); f[sp[i]].im = (int16_t)(ss[i] * sm); }
  zo_ifft128(f, t);
  memcpy(out640, t, sizeof(t));
  memcpy(out640 + 128, t, sizeof(t));
  memcpy(out640 + 256, t, 64 * sizeof(zo_c16));
  static const uint8_t pos[64] = {0, 1, 0, 0, 1, 1, 0, 1, 0, 1, 0, 0, 0, 0, 0, 1, 1, 0, 0, 1, 0, 1, 0, 1, 1, 1, 1, 0, 0, 0, 0, 0,
                                  0, 0, 0, 0, 0, 0, 1, 1, 0, 0, 1, 1, 0, 1, 0, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1, 0, 1, 0, 1, 1, 1, 1};
  memset(f, 0, sizeof(f));
  for (int i = 1; i <= 26; i++) f[i].re = pos[i] ? lm : (int16_t)-lm;
  for (int i = 38; i < 64; i++) f[i + 64].re = pos[i] ? lm : (int16_t)-lm;
  zo_ifft128(f, t);
  zo_c16* l = out640 + 320;
  memcpy(l + 64, t, sizeof(t));
  memcpy(l + 192, t, sizeof(t));
  memcpy(l, l + 256, 64 * sizeof(zo_c16));
}

/* map_ofdm (map_ofdm.blk:63-107) + ifft (ifft.blk:35-52): 48 subcarriers (GetData order) and
   the pilots of symbol k (allPilots index 127 for k = 0, then 0, 1, ...) -> 160 samples */
void zo_tx_symbol(const zo_c16* sub48, int k, zo_c16* out160) {
  const int idx = k == 0 ? 127 : (k - 1) % 127;
  const int16_t B = 10720;
  const int neg = zo_pilot_sign(idx) == -1;
  const int16_t p = neg ? (int16_t)-B : B;
  zo_c16 pil[4] = {{p, 0}, {(int16_t)-p, 0}, {p, 0}, {p, 0}};  /* allPilots, :40-49 */
  zo_c16 e[64];
  memset(e, 0, sizeof(e));
  for (int i = 0; i < 48; i++) {
    static const int bins[48] = {38, 39, 40, 41, 42, 44, 45, 46, 47, 48, 49, 50, 51, 52, 53, 54, 55, 56,
                                 58, 59, 60, 61, 62, 63, 1, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 13, 14, 15,
                                 16, 17, 18, 19, 20, 22, 23, 24, 25, 26};
    e[(bins[i] + 32) & 63] = sub48[i];           /* emitted index = carrier + 32 mod 64 */
  }
  e[(43 + 32) & 63] = pil[2];
  e[(57 + 32) & 63] = pil[3];
  e[(7 + 32) & 63] = pil[0];
  e[(21 + 32) & 63] = pil[1];
  zo_c16 sym[128], t[128];
  memset(sym, 0, sizeof(sym));
  memcpy(sym + 96, e, 32 * sizeof(zo_c16));
  memcpy(sym, e + 32, 32 * sizeof(zo_c16));
  zo_ifft128(sym, t);
  memcpy(out160 + 32, t, sizeof(t));
  memcpy(out160, t + 96, 32 * sizeof(zo_c16));
}

/* transmitter() on one packet: input = 3 PLCP header bytes (emitHeader) + len-4 payload bytes.
   Writes 640 + 160 * (1 + nsym) samples to out (capacity max_out), returns their number. */
int zo_tx_packet(const uint8_t* in, int nin, zo_c16* out, int max_out) {
  if (nin < 3) return -1;
  zo_hdr h;
  uint8_t hb[4] = {in[0], in[1], in[2], 0};
  zo_parse_header(hb, &h);
  const int plen = h.len - 4;
  if (plen < 0 || 3 + plen > nin) return -1;
  const int nd = zo_ndbps(h.modulation, h.coding);
  const int nsym = ((16 + plen * 8 + 32 + 6) + nd - 1) / nd;
  const int total = 640 + 160 * (1 + nsym);
  if (total > max_out) return -1;
  zo_tx_preamble(out);
  zo_c16 sub[48];
  zo_tx_signal_from_bits(in, sub);
  zo_tx_symbol(sub, 0, out + 640);
  zo_c16* d = (zo_c16*)malloc(sizeof(zo_c16) * 48 * (size_t)nsym);
  zo_tx_data_symbols(in + 3, plen, h.modulation, h.coding, d, nsym);
  for (int k = 0; k < nsym; k++) zo_tx_symbol(d + 48 * k, k + 1, out + 640 + 160 * (1 + k));
  free(d);
  return total;
}
