/*
 * ORACLE — test infrastructure only (see ziria_oracle.h).  Scalar, deliberately plain C:
 * every routine restates one reference routine in the most literal form, so that it can
 * be read side by side with the cited reference lines.  Not part of the product.
 */
#include "ziria_oracle.h"
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------ */
/* int16 helpers: SSE2 adds/subs_epi16 saturate; XOR with 0xFFFF is ~x = -x-1.          */
static inline int16_t sat16(int32_t x) { return (int16_t)(x > 32767 ? 32767 : (x < -32768 ? -32768 : x)); }
static inline int16_t inv16(int16_t x) { return (int16_t)~x; }
static inline zo_c16 cadd(zo_c16 a, zo_c16 b) { zo_c16 r = {sat16(a.re + b.re), sat16(a.im + b.im)}; return r; }
static inline zo_c16 csub(zo_c16 a, zo_c16 b) { zo_c16 r = {sat16(a.re - b.re), sat16(a.im - b.im)}; return r; }
static inline zo_c16 cshr2(zo_c16 a) { zo_c16 r = {(int16_t)(a.re >> 2), (int16_t)(a.im >> 2)}; return r; }

/* mul_shiftx(a, b, 15): csrc/sora_ext_lib_fft.hpp:42-67.  _mm_madd_epi16 sums two exact
   32-bit products with 32-bit wrap; srai 15; keep low 16 bits. */
static inline zo_c16 mul_shift(zo_c16 a, int16_t bre, int16_t bim) {
  int64_t re = (int64_t)a.re * bre + (int64_t)a.im * (int16_t)~bim;
  int64_t im = (int64_t)a.re * bim + (int64_t)a.im * bre;
  int32_t re32 = (int32_t)(uint32_t)re, im32 = (int32_t)(uint32_t)im;
  zo_c16 r = {(int16_t)(re32 >> 15), (int16_t)(im32 >> 15)};
  return r;
}
/* mul_jx: csrc/sora_ext_lib_fft.hpp:98-108 — swap re/im, then XOR low half: (~im, re). */
static inline zo_c16 mul_j(zo_c16 a) { zo_c16 r = {inv16(a.im), a.re}; return r; }

/* twFFTLUT{N}_{k}[n] (csrc/sora_ext_lib_fft_coeffs.hpp:53-78, 298-359):
   clamp(round(32768 e^{-j 2 pi k n / N}), -32767, 32767) per component.  Checked against
   the reference brick's FFT outputs (tests/test_oracle_golden.py). */
void zo_twiddle(int N, int k, int n, int16_t* re, int16_t* im) {
  double ang = -2.0 * M_PI * (double)k * (double)n / (double)N;
  double r = floor(32768.0 * cos(ang) + 0.5), i = floor(32768.0 * sin(ang) + 0.5);
  if (r > 32767) r = 32767; if (r < -32767) r = -32767;
  if (i > 32767) i = 32767; if (i < -32767) i = -32767;
  *re = (int16_t)r; *im = (int16_t)i;
}

/* FFTSSE<N>: csrc/fft_r4difx.hpp:54-97 (radix-4 DIF stage, in place) */
static void fft_stage(zo_c16* x, int N) {
  for (int n = 0; n < N / 4; n++) {
    zo_c16 a = cshr2(x[n]), b = cshr2(x[n + N / 4]), c = cshr2(x[n + N / 2]), d = cshr2(x[n + 3 * N / 4]);
    zo_c16 ac = cadd(a, c), bd = cadd(b, d), a_c = csub(a, c), b_d = csub(b, d);
    int16_t tr, ti;
    x[n] = cadd(ac, bd);
    zo_twiddle(N, 2, n, &tr, &ti);
    x[n + N / 4] = mul_shift(csub(ac, bd), tr, ti);
    zo_c16 jb = mul_j(b_d);
    zo_twiddle(N, 1, n, &tr, &ti);
    x[n + N / 2] = mul_shift(csub(a_c, jb), tr, ti);
    zo_twiddle(N, 3, n, &tr, &ti);
    x[n + 3 * N / 4] = mul_shift(cadd(a_c, jb), tr, ti);
  }
}
/* FFTSSEEx<4>: csrc/fft_r4difx.hpp:111-140 (4-point DFT with XOR-as-negate) */
static void fft4(zo_c16* x) {
  zo_c16 y0 = cshr2(x[0]), y1 = cshr2(x[1]), y2 = cshr2(x[2]), y3 = cshr2(x[3]);
  int16_t a0 = sat16(y0.re + y2.re), a1 = sat16(y0.im + y2.im);
  int16_t a2 = sat16(y1.re + y3.re), a3 = sat16(y1.im + y3.im);
  int16_t L4 = sat16(y0.re + inv16(y2.re)), L5 = sat16(y0.im + inv16(y2.im));
  int16_t L6 = sat16(y1.re + inv16(y3.re));
  int16_t L7 = inv16(sat16(y1.im + inv16(y3.im)));
  x[0].re = sat16(a0 + a2);           x[0].im = sat16(a1 + a3);
  x[1].re = sat16(inv16(a2) + a0);    x[1].im = sat16(inv16(a3) + a1);
  x[2].re = sat16(inv16(L7) + L4);    x[2].im = sat16(inv16(L6) + L5);
  x[3].re = sat16(L4 + L7);           x[3].im = sat16(L5 + L6);
}
static int bitrev6(int i) {
  int r = 0;
  for (int b = 0; b < 6; b++) r |= ((i >> b) & 1) << (5 - b);
  return r;
}
/* FFT<64>/FFTSafe<64>: csrc/fft_r4difx.hpp:220-237; output map bFFT64LUTMap
   (csrc/sora_ext_lib_fft_coeffs.hpp:15090-15094) = 6-bit bit reversal. */
void zo_fft64(const zo_c16* in, zo_c16* out) {
  zo_c16 x[64];
  memcpy(x, in, sizeof(x));
  fft_stage(x, 64);
  for (int q = 0; q < 4; q++) {
    fft_stage(x + 16 * q, 16);
    for (int r = 0; r < 4; r++) fft4(x + 16 * q + 4 * r);
  }
  for (int i = 0; i < 64; i++) out[i] = x[bitrev6(i)];
}

/* ---- FFTSafe<N> for every size __ext_sora_fft dispatches (csrc/sora_ext_lib.cpp:2672-2812) */
static inline zo_c16 cshr3(zo_c16 a) { zo_c16 r = {(int16_t)(a.re >> 3), (int16_t)(a.im >> 3)}; return r; }
static inline zo_c16 cinv(zo_c16 a) { zo_c16 r = {inv16(a.re), inv16(a.im)}; return r; }
static inline zo_c16 tw(int N, int k, int n) { zo_c16 t; zo_twiddle(N, k, n, &t.re, &t.im); return t; }
static inline zo_c16 mul_c(zo_c16 a, zo_c16 b) { return mul_shift(a, b.re, b.im); }

/* FFTSSE_3<N>: csrc/sora_ext_lib_fft.hpp:111-171 (radix-3 DIF stage, input >> 2, the
   rotations e^{-j2pi/3}, e^{-j4pi/3} as (-16384, -+28378), outputs in natural thirds) */
static void fft_stage3(zo_c16* x, int N) {
  const zo_c16 k1 = {-16384, -28378}, k2 = {-16384, 28378};
  const int M = N / 3;
  for (int n = 0; n < M; n++) {
    zo_c16 a = cshr2(x[n]), b = cshr2(x[n + M]), c = cshr2(x[n + 2 * M]);
    zo_c16 bk1 = mul_c(b, k1), bk2 = mul_c(b, k2), ck1 = mul_c(c, k1), ck2 = mul_c(c, k2);
    x[n] = cadd(cadd(a, b), c);
    x[n + M] = mul_c(cadd(cadd(a, bk1), ck2), tw(N, 1, n));
    x[n + 2 * M] = mul_c(cadd(cadd(a, bk2), ck1), tw(N, 2, n));
  }
}
/* FFTSSE_5<N>: csrc/sora_ext_lib_fft.hpp:253-349 (radix-5 DIF stage, input >> 3) */
static void fft_stage5(zo_c16* x, int N) {
  const zo_c16 k1 = {10126, -31164}, k2 = {-26510, -19261}, k3 = {-26510, 19261}, k4 = {10126, 31164};
  const int M = N / 5;
  for (int n = 0; n < M; n++) {
    zo_c16 a = cshr3(x[n]), b = cshr3(x[n + M]), c = cshr3(x[n + 2 * M]), d = cshr3(x[n + 3 * M]),
           e = cshr3(x[n + 4 * M]);
    zo_c16 bk1 = mul_c(b, k1), bk2 = mul_c(b, k2), bk3 = mul_c(b, k3), bk4 = mul_c(b, k4);
    zo_c16 ck1 = mul_c(c, k1), ck2 = mul_c(c, k2), ck3 = mul_c(c, k3), ck4 = mul_c(c, k4);
    zo_c16 dk1 = mul_c(d, k1), dk2 = mul_c(d, k2), dk3 = mul_c(d, k3), dk4 = mul_c(d, k4);
    zo_c16 ek1 = mul_c(e, k1), ek2 = mul_c(e, k2), ek3 = mul_c(e, k3), ek4 = mul_c(e, k4);
    x[n] = cadd(cadd(cadd(a, b), cadd(c, d)), e);
    x[n + M] = mul_c(cadd(cadd(cadd(a, bk1), cadd(ck2, dk3)), ek4), tw(N, 1, n));
    x[n + 2 * M] = mul_c(cadd(cadd(cadd(a, bk2), cadd(ck4, dk1)), ek3), tw(N, 2, n));
    x[n + 3 * M] = mul_c(cadd(cadd(cadd(a, bk3), cadd(ck1, dk4)), ek2), tw(N, 3, n));
    x[n + 4 * M] = mul_c(cadd(cadd(cadd(a, bk4), cadd(ck3, dk2)), ek1), tw(N, 4, n));
  }
}
/* FFTSSEEx<8>: csrc/fft_r4difx.hpp:142-218, the SSE lane sequence restated per complex
   value: input >> 3; d = x[k] - x[k+4], s = x[k] + x[k+4]; the lower half rotates d2, d3
   by (im, ~re), combines, multiplies by (32767,0), (23169,-23169), (32767,0),
   (-23169,-23169) and finishes with XOR-as-negate pairs; the upper half is a 4-point DFT
   of s with the same pairing.  Output positions 0..3 = the upper half, 4..7 = the lower. */
static void fft8(zo_c16* x) {
  zo_c16 d[4], s[4], e[4], f[4], t[4], u[4];
  for (int k = 0; k < 4; k++) {
    zo_c16 a = cshr3(x[k]), b = cshr3(x[k + 4]);
    d[k] = csub(a, b);
    s[k] = cadd(a, b);
  }
  zo_c16 m2 = {d[2].im, inv16(d[2].re)}, m3 = {d[3].im, inv16(d[3].re)};
  e[0] = cadd(d[0], m2); e[1] = cadd(d[1], m3); e[2] = cadd(cinv(m2), d[0]); e[3] = cadd(cinv(m3), d[1]);
  const zo_c16 w[4] = {{32767, 0}, {23169, -23169}, {32767, 0}, {-23169, -23169}};
  for (int k = 0; k < 4; k++) f[k] = mul_c(e[k], w[k]);
  t[0] = cadd(s[0], s[2]); t[1] = cadd(s[1], s[3]); t[2] = cadd(cinv(s[2]), s[0]); t[3] = cadd(cinv(s[3]), s[1]);
  u[0] = t[0]; u[1] = t[1]; u[2] = t[2]; u[3].re = t[3].im; u[3].im = inv16(t[3].re);
  x[0] = cadd(u[0], u[1]); x[1] = cadd(cinv(u[1]), u[0]); x[2] = cadd(u[2], u[3]); x[3] = cadd(cinv(u[3]), u[2]);
  x[4] = cadd(f[0], f[1]); x[5] = cadd(f[0], cinv(f[1])); x[6] = cadd(f[2], f[3]); x[7] = cadd(f[2], cinv(f[3]));
}
/* The radix of the first stage of FFTSSEEx<N>: the template specialisations route these
   sizes to FFTSSE_3W (csrc/sora_ext_lib_fft.hpp:190-251) and FFTSSE_5W (:366-430); every
   other size takes the generic radix-4 FFTSSEEx (csrc/fft_r4difx.hpp:99-109); 4 and 8 are
   the base cases (:111-218). */
int zo_fft_radix(int N) {
  switch (N) {
    case 4: case 8: return 0;
    case 12: case 24: case 36: case 72: case 108: case 216: case 324: case 648: case 972: return 3;
    case 60: case 120: case 180: case 300: case 360: case 540: case 600: case 900: case 1080: return 5;
    default: return 4;
  }
}
static void fft_ex(zo_c16* x, int N) {
  const int r = zo_fft_radix(N);
  if (r == 0) { if (N == 4) fft4(x); else fft8(x); return; }
  if (r == 4) fft_stage(x, N); else if (r == 3) fft_stage3(x, N); else fft_stage5(x, N);
  for (int q = 0; q < r; q++) fft_ex(x + q * (N / r), N / r);
}
/* Frequency index held at each position after fft_ex (the reference's bFFT{N}LUTMap is its
   inverse, csrc/sora_ext_lib_fft_coeffs.hpp:15053-15260): a radix-4 stage leaves residues
   0, 2, 1, 3 in its quarters, radix 3 / 5 stages leave them in order, the base cases are
   bit-reversed. */
void zo_fft_freq_of_pos(int N, int* idx) {
  const int r = zo_fft_radix(N);
  if (r == 0) {
    for (int p = 0; p < N; p++) idx[p] = N == 4 ? ((p & 1) << 1 | (p >> 1)) : ((p & 1) << 2 | (p & 2) | (p >> 2));
    return;
  }
  const int M = N / r;
  int* sub = (int*)malloc(sizeof(int) * M);
  zo_fft_freq_of_pos(M, sub);
  static const int res4[4] = {0, 2, 1, 3};
  for (int q = 0; q < r; q++)
    for (int p = 0; p < M; p++) idx[q * M + p] = r * sub[p] + (r == 4 ? res4[q] : q);
  free(sub);
}
int zo_fft_supported(int N) {
  static const int sz[] = {16, 32, 64, 128, 256, 512, 1024, 2048, 12, 24, 36, 48, 60, 72, 96, 108, 120, 144,
                           180, 192, 216, 240, 288, 300, 324, 360, 384, 432, 480, 540, 576, 600, 648, 720, 768,
                           864, 900, 960, 972, 1080, 1152, 1200};
  for (unsigned i = 0; i < sizeof(sz) / sizeof(sz[0]); i++) if (sz[i] == N) return 1;
  return 0;
}
/* FFTSafe<N> (csrc/fft_r4difx.hpp:220-237): the stages on a copy, then out[f] = the
   position holding frequency f.  Returns 0, or -1 for a size the reference rejects. */
int zo_fft_n(int N, const zo_c16* in, zo_c16* out) {
  if (!zo_fft_supported(N)) return -1;
  zo_c16* x = (zo_c16*)malloc(sizeof(zo_c16) * N);
  int* idx = (int*)malloc(sizeof(int) * N);
  memcpy(x, in, sizeof(zo_c16) * N);
  fft_ex(x, N);
  zo_fft_freq_of_pos(N, idx);
  for (int p = 0; p < N; p++) out[idx[p]] = x[p];
  free(x); free(idx);
  return 0;
}

/* __ext_v_shift_right_complex16 (csrc/sora_ext_lib.cpp:1979-1995): whole groups of 4
   complex values use _mm_srai_epi16 (arithmetic, counts > 15 fill with the sign); the
   remaining values use unum16 >> shift (logical). */
int zo_v_shift_right_complex16(zo_c16* z, const zo_c16* x, int len, int shift) {
  const int16_t* P = (const int16_t*)x;
  int16_t* Q = (int16_t*)z;
  int nvec = (len / 4) * 8;
  for (int i = 0; i < 2 * len; i++) {
    if (i < nvec) Q[i] = (int16_t)((shift < 0 || shift > 15) ? (P[i] < 0 ? -1 : 0) : (P[i] >> shift));
    else Q[i] = (int16_t)((shift < 0 || shift > 15) ? 0 : ((uint16_t)P[i] >> shift));
  }
  return 0;
}

/* ------------------------------------------------------------------------------------ */
/* GetData.blk:24-35: bins 38..42, 44..56, 58..63, 1..6, 8..20, 22..26 */
void zo_get_data(const zo_c16* s, zo_c16* o) {
  static const int seg[6][2] = {{38, 5}, {44, 13}, {58, 6}, {1, 6}, {8, 13}, {22, 5}};
  int k = 0;
  for (int g = 0; g < 6; g++)
    for (int i = 0; i < seg[g][1]; i++) o[k++] = s[seg[g][0] + i];
}
/* DemapLimit.blk:22-63 with v_shift_right_complex16(.., 0) (sora_ext_lib.cpp:1979-1995):
   clip re/im to [-128,127], then map negatives to 256+v (u8 LUT index). */
void zo_demap_limit(const zo_c16* in, int n, zo_c16* out) {
  for (int i = 0; i < n; i++) {
    int re = in[i].re, im = in[i].im;
    re = re < -128 ? -128 : (re > 127 ? 127 : re);
    im = im < -128 ? -128 : (im > 127 ? 127 : im);
    out[i].re = (int16_t)(re < 0 ? 256 + re : re);
    out[i].im = (int16_t)(im < 0 ? 256 + im : im);
  }
}
/* Demap LUTs, code/WiFi/const.blk:74-150, one digit per entry. */
static const char* const LUT_STR[4] = {
  "4444444445555555556666666666666777777777777777777777777777777777"
  "7777777777777777777777777777777777777777777777777777777777777777"
  "0000000000000000000000000000000000000000000000000000000000000000"
  "0000000000000000000000000000000000111111111111122222222233333333",
  "7777777777777777777777777777777777777777777777777777777766655544"
  "3322111000000000000000000000000000000000000000000000000000000000"
  "0000000000000000000000000000000000000000000000000000000000111223"
  "3445556667777777777777777777777777777777777777777777777777777777",
  "7777777777777777777777777777777777777777777777777777777766655433"
  "2211100000000000000000000000000000000000000000000000000000000000"
  "0000000000000000000000000000000000000000000000000000000000001112"
  "2334556667777777777777777777777777777777777777777777777777777777",
  "0000000000000000000000000111223445566677777777777777777777777777"
  "7777777777777777777777766654433221100000000000000000000000000000"
  "0000000000000000000000000000001122334456667777777777777777777777"
  "7777777777777777777777777776665544322111000000000000000000000000",
};
const uint8_t* zo_lut(int which) {
  static uint8_t t[4][256];
  static int init = 0;
  if (!init) {
    for (int w = 0; w < 4; w++)
      for (int i = 0; i < 256; i++) t[w][i] = (uint8_t)(LUT_STR[w][i] - '0');
    init = 1;
  }
  return t[which];
}
int zo_ncbps(int mod) { return mod == 0 ? 48 : mod == 1 ? 96 : mod == 2 ? 192 : 288; }
/* transmitter.blk:39-46 */
int zo_ndbps(int mod, int coding) {
  int nc = zo_ncbps(mod);
  return coding == 0 ? nc / 2 : coding == 1 ? nc * 2 / 3 : nc * 3 / 4;
}
/* DemapBPSK/QPSK/QAM16/QAM64.blk:22-33 — symbol is the DemapLimit output (u8 index). */
int zo_demap(int mod, const zo_c16* lim, int8_t* soft) {
  const uint8_t *B = zo_lut(0), *Q16 = zo_lut(1), *Q2 = zo_lut(2), *Q3 = zo_lut(3);
  int k = 0;
  for (int i = 0; i < 48; i++) {
    int re = lim[i].re & 0xFF, im = lim[i].im & 0xFF;
    switch (mod) {
      case 0: soft[k++] = (int8_t)B[re]; break;
      case 1: soft[k++] = (int8_t)B[re]; soft[k++] = (int8_t)B[im]; break;
      case 2: soft[k++] = (int8_t)B[re]; soft[k++] = (int8_t)Q16[re];
              soft[k++] = (int8_t)B[im]; soft[k++] = (int8_t)Q16[im]; break;
      default: soft[k++] = (int8_t)B[re]; soft[k++] = (int8_t)Q2[re]; soft[k++] = (int8_t)Q3[re];
               soft[k++] = (int8_t)B[im]; soft[k++] = (int8_t)Q2[im]; soft[k++] = (int8_t)Q3[im];
    }
  }
  return k;
}
/* Deinterleave{BPSK,QPSK,QAM16,QAM64}.blk: out[k] = in[p(k)], p = the 802.11a interleaver
   index map (transmitter/interleaving.blk:38-58) — equality with the .blk tables is
   checked against tests/golden/deinterleave_perm.npz. */
int zo_deint_src(int mod, int k) {
  int N = zo_ncbps(mod), nbpsc = N / 48;
  int s = nbpsc / 2 > 1 ? nbpsc / 2 : 1;
  int i = (N / 16) * (k % 16) + k / 16;
  return s * (i / s) + (i + N - (16 * i) / N) % s;
}
void zo_deinterleave(int mod, const int8_t* in, int8_t* out) {
  int N = zo_ncbps(mod);
  for (int k = 0; k < N; k++) out[k] = in[zo_deint_src(mod, k)];
}

/* ------------------------------------------------------------------------------------ */
/* Viterbi.  Branch metric of VIT_MA / VIT_MB (csrc/viterbilut.h:111-285): entry
   [soft*8 + 2g + b][j] is the metric of branch b (0: from p0=s>>1, 1: from p1=p0|32) into
   new state s = 16g + j for soft value `soft`; expected code bit from encoding.blk:92-109
   (A: x^p1^p2^p4^p5, B: x^p0^p1^p2^p5); metric e ? 14-2v : 2v. */
static inline int bit_(int v, int b) { return (v >> b) & 1; }
static inline int exp_a(int p, int x) { return x ^ bit_(p, 1) ^ bit_(p, 2) ^ bit_(p, 4) ^ bit_(p, 5); }
static inline int exp_b(int p, int x) { return x ^ bit_(p, 0) ^ bit_(p, 1) ^ bit_(p, 2) ^ bit_(p, 5); }
static inline int bm(int v, int e) { return e ? 14 - 2 * v : 2 * v; }
int zo_vit_lut(int which, int soft, int k, int j) {
  int g = k >> 1, b = k & 1, s = 16 * g + j, p = (s >> 1) | (b ? 32 : 0), x = s & 1;
  return bm(soft, which == 0 ? exp_a(p, x) : exp_b(p, x));
}

/* one trellis step = computeNextACSState / 1-input BranchACS
   (csrc/viterbicore.hpp:105-147, 241-265, 343-390).  use: 3 = A and B, 1 = A only, 2 = B only */
static void acs(const uint8_t* m, uint8_t* nm, int a, int b, int use) {
  for (int s = 0; s < 64; s++) {
    int p0 = s >> 1, p1 = p0 | 32, x = s & 1;
    int b0 = 0, b1 = 0;
    if (use & 1) { b0 += bm(a, exp_a(p0, x)); b1 += bm(a, exp_a(p1, x)); }
    if (use & 2) { int v = (use == 2) ? a : b; b0 += bm(v, exp_b(p0, x)); b1 += bm(v, exp_b(p1, x)); }
    int r0 = ((m[p0] + b0) & 0xFF) & 0xFE;   /* _mm_add_epi8 wraps; AND ALL_INVERSE_ONE */
    int r1 = ((m[p1] + b1) & 0xFF) | 1;      /* OR ALL_ONE */
    nm[s] = (uint8_t)(r0 < r1 ? r0 : r1);    /* _mm_min_epu8 */
  }
}
static uint64_t lsb_word(const uint8_t* m) {
  uint64_t w = 0;
  for (int s = 0; s < 64; s++) w |= (uint64_t)(m[s] & 1) << s;
  return w;
}
/* normalize: csrc/viterbicore.hpp:149-168 */
static void normalize(uint8_t* m) {
  int mn = 255;
  for (int s = 0; s < 64; s++) if (m[s] < mn) mn = m[s];
  mn &= 0xFE;
  for (int s = 0; s < 64; s++) m[s] = (uint8_t)(m[s] - mn);
}
/* traceback: csrc/viterbicore.hpp:170-239 (SSE2 hmin16: signed int16 key). */
static void traceback(const uint8_t* m, const uint64_t* surv, uint32_t col, uint8_t* out,
                      uint32_t output_bits, uint32_t lookahead) {
  int best = 0x7FFFFFFF;
  for (int s = 0; s < 64; s++) {
    int key = (int16_t)(uint16_t)((m[s] << 8) | (4 * s));
    if (key < best) best = key;
  }
  int i = (best >> 2) & 0x7F;
  uint32_t t = col;
  for (uint32_t k = 0; k < lookahead; k++) {
    t--;
    i = (i >> 1) & 0x3F;
    i |= (int)((surv[t] >> i) & 1) << 6;
  }
  uint32_t nbytes = output_bits >> 3;
  for (uint32_t byte = nbytes; byte-- > 0;) {
    int oc = 0;
    for (int j = 0; j < 8; j++) {
      oc = (oc << 1) | ((i >> 6) & 1);
      t--;
      i = (i >> 1) & 0x3F;
      i |= (int)((surv[t] >> i) & 1) << 6;
    }
    out[byte] = (uint8_t)oc;
  }
}

/* __ext_viterbi_brick_init_fast: csrc/sora_ext_viterbi.cpp:48-63 ; Reset: viterbicore.hpp:329-338 */
int zo_vit_init(zo_vit* v, int frame_len, int code_rate, int depth) {
  if (!v->surv) {
    v->cap = 40000 + 8;                       /* TRELLIS_MAX = 5000*8 (:39) */
    v->surv = (uint64_t*)calloc(v->cap, sizeof(uint64_t));
    if (!v->surv) return -1;
  }
  v->m[0] = 0;
  for (int s = 1; s < 64; s++) v->m[s] = 48;  /* ALL_INIT0 / ALL_INIT */
  v->surv[0] = 0;
  v->tr = 0; v->ob = 0;
  v->frame_len = frame_len; v->code_rate = code_rate; v->depth = depth;
  return 0;
}
void zo_vit_free(zo_vit* v) { free(v->surv); v->surv = 0; }

static void step(zo_vit* v, int a, int b, int use) {
  uint8_t nm[64];
  acs(v->m, nm, a, b, use);
  memcpy(v->m, nm, 64);
  v->tr++;
  if (v->tr < v->cap) v->surv[v->tr] = lsb_word(v->m);
}
/* __ext_viterbi_brick_decode_fast: csrc/sora_ext_viterbi.cpp:66-153 */
int zo_vit_decode(zo_vit* v, const int8_t* soft, int n, uint8_t* out) {
  const int prefix = 6, look = 24;
  const uint8_t* in = (const uint8_t*)soft;
  const uint8_t* end = in + n;
  uint32_t total_bytes = 0;
  uint8_t tmp[4096];
  while (in < end) {
    /* the brick's trellis has TRELLIS_MAX = 40000 columns (sora_ext_viterbi.cpp:39) and it
       writes past them; here (as in the engine) groups that do not fit are not consumed */
    const uint32_t steps = v->code_rate == 0 ? 1u : v->code_rate == 1 ? 2u : 3u;
    if (v->tr + steps >= 40000u) break;
    if (v->code_rate == 0) { step(v, in[0], in[1], 3); in += 2; }
    else if (v->code_rate == 2) { step(v, in[0], in[1], 3); step(v, in[2], 0, 1); step(v, in[3], 0, 2); in += 4; }
    else if (v->code_rate == 1) { step(v, in[0], in[1], 3); step(v, in[2], 0, 1); in += 3; }
    else break;
    uint32_t tr = v->tr;
    if ((tr & 7) == 0) {
      normalize(v->m);
      if (tr < v->cap) v->surv[tr] = lsb_word(v->m);   /* LSBs unchanged by normalize */
    }
    uint32_t output_count = 0, lookahead = 0;
    uint32_t tr_end = (uint32_t)v->frame_len * 8 + prefix;
    if (tr >= tr_end) {
      output_count = tr_end - v->ob - prefix;
      lookahead = tr - tr_end;
    } else if (tr >= v->ob + (uint32_t)v->depth + look + prefix) {
      uint32_t remain = (tr - (v->ob + v->depth + look + prefix)) % 8;
      output_count = v->depth;
      lookahead = look + remain;
    }
    if (output_count) {
      traceback(v->m, v->surv, tr, tmp, output_count, lookahead);
      v->ob += output_count;
      for (uint32_t k = 0; k < output_count / 8; k++) out[total_bytes++] = tmp[k];
    }
  }
  return (int)(total_bytes * 8);
}

/* __ext_viterbiSig11a_brick_decode_fast: csrc/sora_ext_viterbi.cpp:176-194 ->
   Viterbi_sig11 csrc/viterbicore.hpp:272-315 */
void zo_vit_sig(const int8_t* soft48, uint8_t* bits4) {
  uint8_t m[64];
  uint64_t surv[25];
  m[0] = 0;
  for (int s = 1; s < 64; s++) m[s] = 48;
  surv[0] = 0;
  for (int t = 1; t <= 24; t++) {
    uint8_t nm[64];
    acs(m, nm, (uint8_t)soft48[2 * t - 2], (uint8_t)soft48[2 * t - 1], 3);
    memcpy(m, nm, 64);
    if ((t & 7) == 0) normalize(m);
    surv[t] = lsb_word(m);
  }
  normalize(m);
  traceback(m, surv, 24, bits4, 24, 0);
  uint32_t w = (uint32_t)bits4[0] | ((uint32_t)bits4[1] << 8) | ((uint32_t)bits4[2] << 16) |
               ((uint32_t)bits4[3] << 24);
  w >>= 6;                                      /* *((unum32*)bit) >>= 6  (:191) */
  bits4[0] = (uint8_t)w; bits4[1] = (uint8_t)(w >> 8); bits4[2] = (uint8_t)(w >> 16);
  bits4[3] = (uint8_t)(w >> 24);
}

/* ------------------------------------------------------------------------------------ */
static inline int getbit(const uint8_t* b, int k) { return (b[k >> 3] >> (k & 7)) & 1; }
static inline void setbit(uint8_t* b, int k, int v) {
  if (v) b[k >> 3] |= (uint8_t)(1 << (k & 7)); else b[k >> 3] &= (uint8_t)~(1 << (k & 7));
}
/* parsePLCPHeader: code/WiFi/transmitter/parsePLCPHeader.blk:119-213 (after
   ViterbiSig11a.blk:37 zeroes bits 18..23) */
void zo_parse_header(const uint8_t* hb, zo_hdr* h) {
  int b0 = getbit(hb, 0), b1 = getbit(hb, 1), b2 = getbit(hb, 2), b3 = getbit(hb, 3);
  int code = b0 | (b1 << 1) | (b2 << 2) | (b3 << 3);
  switch (code) {
    case 0xB: h->modulation = 0; h->coding = 0; break;   /* 1101 */
    case 0xF: h->modulation = 0; h->coding = 2; break;   /* 1111 */
    case 0xA: h->modulation = 1; h->coding = 0; break;   /* 0101 */
    case 0xE: h->modulation = 1; h->coding = 2; break;   /* 0111 */
    case 0x9: h->modulation = 2; h->coding = 0; break;   /* 1001 */
    case 0xD: h->modulation = 2; h->coding = 2; break;   /* 1011 */
    case 0x8: h->modulation = 3; h->coding = 1; break;   /* 0001 */
    case 0xC: h->modulation = 3; h->coding = 2; break;   /* 0011 */
    default: h->modulation = 0; h->coding = 0;
  }
  int len = 0, bb = 1;
  for (int j = 5; j < 17; j++) { if (getbit(hb, j)) len += bb; bb *= 2; }
  h->err = 0;
  if (len > 2048) { h->err = 1; len = 2048; }
  h->len = len;
  int p = 0;
  for (int k = 0; k < 24; k++) p ^= getbit(hb, k);
  if (p) h->err = 1;
  p = 0;
  for (int j = 2; j < 8; j++) p |= getbit(hb, 16 + j);
  if (p) h->err = 1;
}

/* update_crc_generic (crc.blk:41-73) literally, on bit arrays, base32 = 0x04C11DB7. */
static const uint8_t BASE32[33] = {1,0,0,0,0,0,1,0,0,1,1,0,0,0,0,0,1,0,0,0,1,1,1,0,1,1,0,1,1,0,1,1,1};
static void update_crc_generic(const uint8_t* x, uint8_t* st) {
  uint8_t out[40] = {0}, ss[8];
  for (int i = 0; i < 8; i++) ss[i] = st[i] ^ x[i];
  for (int i = 0; i < 8; i++) {
    if (ss[i]) {
      for (int j = 0; j < 31; j++) out[i + 1 + j] ^= BASE32[1 + j];
      for (int j = 0; j < 8 - i - 1; j++) ss[i + 1 + j] ^= BASE32[1 + j];
    }
  }
  uint8_t ns[32];
  for (int k = 0; k < 24; k++) ns[k] = st[8 + k];
  for (int k = 0; k < 8; k++) ns[24 + k] = ss[k];
  for (int k = 0; k < 32; k++) st[k] = ns[k] ^ out[8 + k];
}
/* crc_template.blk:29-70 with pad=false: CRC state bits after inversion, packed
   LSB-first (bits_to_int8) into a little-endian u32. */
uint32_t zo_crc32_bits(const uint8_t* bytes, int nbytes) {
  uint8_t st[32];
  for (int k = 0; k < 32; k++) st[k] = 1;
  for (int n = 0; n < nbytes; n++) {
    uint8_t x[8];
    for (int j = 0; j < 8; j++) x[j] = (bytes[n] >> j) & 1;
    update_crc_generic(x, st);
  }
  uint32_t w = 0;
  for (int k = 0; k < 32; k++) w |= (uint32_t)(st[k] ^ 1) << k;
  return w;
}
/* descrambler (Decode.blk:36-43 + scramble.blk:28-44) then crc(len-4,false)+check_crc
   (receiver.blk:47-48, crc.blk:85-118). */
int zo_descramble_crc(const uint8_t* dec, int len, uint8_t* payload) {
  int st[7];
  for (int k = 0; k < 7; k++) st[k] = getbit(dec, 9 + k);
  int nbits = len * 8;
  uint8_t* tmp = (uint8_t*)calloc((size_t)len + 1, 1);
  for (int k = 0; k < nbits; k++) {
    int t = st[3] ^ st[0];
    for (int q = 0; q < 6; q++) st[q] = st[q + 1];
    st[6] = t;
    setbit(tmp, k, getbit(dec, 16 + k) ^ t);
  }
  int plen = len - 4;
  if (plen < 0) plen = 0;
  memcpy(payload, tmp, (size_t)plen);
  uint32_t c = zo_crc32_bits(tmp, plen);
  uint32_t rx = (uint32_t)tmp[plen] | ((uint32_t)tmp[plen + 1] << 8) | ((uint32_t)tmp[plen + 2] << 16) |
                ((uint32_t)tmp[plen + 3] << 24);
  free(tmp);
  return len >= 4 && c == rx;
}

/* receiveBits (receiver.blk:43-54) over frequency-domain data subcarriers. */
static int rx_freq_impl(const zo_c16* sub, int nsym, uint8_t* payload, zo_rx_result* r) {
  memset(r, 0, sizeof(*r));
  if (nsym < 1) return -1;
  zo_c16 lim[48];
  int8_t soft[288], di[288];
  /* DecodePLCP.blk:30-37 */
  zo_demap_limit(sub, 48, lim);
  zo_demap(0, lim, soft);
  zo_deinterleave(0, soft, di);
  uint8_t hb[4] = {0, 0, 0, 0};
  zo_vit_sig(di, hb);
  hb[2] &= 0x03;                       /* ViterbiSig11a.blk:37: bits 18..23 := 0 */
  hb[3] = 0;
  zo_parse_header(hb, &r->h);
  /* Decode.blk:45-60 */
  int mod = r->h.modulation, cod = r->h.coding, len = r->h.len;
  int nc = zo_ncbps(mod), nd = zo_ndbps(mod, cod);
  int need = (16 + 8 * len + 6 + nd - 1) / nd;      /* symbols that hold SERVICE..tail */
  zo_vit v; memset(&v, 0, sizeof(v));
  zo_vit_init(&v, len + 2, cod, 256);
  uint8_t* dec = (uint8_t*)calloc((size_t)len + 16, 1);
  int bits = 0, used = 0;
  for (int k = 0; k < nsym - 1 && bits < (len + 2) * 8; k++) {
    zo_demap_limit(sub + 48 * (1 + k), 48, lim);
    zo_demap(mod, lim, soft);
    zo_deinterleave(mod, soft, di);
    for (int c = 0; c < nc; c += 48) bits += zo_vit_decode(&v, di + c, 48, dec + bits / 8);
    used++;
  }
  zo_vit_free(&v);
  r->nsym_used = 1 + used;
  r->viterbi_bits = bits;
  int ret = (bits >= (len + 2) * 8) ? 0 : -2;
  (void)need;
  r->crc_ok = (ret == 0) ? zo_descramble_crc(dec, len, payload) : 0;
  free(dec);
  return ret;
}
int zo_rx_packet_freq(const zo_c16* sub48, int nsym, uint8_t* payload, zo_rx_result* r) {
  return rx_freq_impl(sub48, nsym, payload, r);
}
/* FFT() (OFDM/FFT.blk:24-30) >>> GetData() >>> receiveBits() */
int zo_rx_packet_time(const zo_c16* sym, int nsym, uint8_t* payload, zo_rx_result* r) {
  zo_c16* sub = (zo_c16*)malloc(sizeof(zo_c16) * 48 * (size_t)(nsym > 0 ? nsym : 1));
  zo_c16 f[64];
  for (int k = 0; k < nsym; k++) {
    zo_fft64(sym + 64 * k, f);
    zo_get_data(f, sub + 48 * k);
  }
  int ret = rx_freq_impl(sub, nsym, payload, r);
  free(sub);
  return ret;
}

/* ------------------------------------------------------------------------------------ */
typedef struct {
  int kind, t, nt, npkts;
  const void* a; const int64_t* off; const int32_t* n;
  const int32_t* fl; const int16_t* cr; uint8_t* out; const int64_t* ooff;
  int stride; zo_rx_result* res;
} job_t;
static void* worker(void* p) {
  job_t* j = (job_t*)p;
  zo_vit v; memset(&v, 0, sizeof(v));
  for (int i = j->t; i < j->npkts; i += j->nt) {
    if (j->kind == 0) {
      zo_vit_init(&v, j->fl[i], j->cr[i], 256);
      zo_vit_decode(&v, (const int8_t*)j->a + j->off[i], j->n[i], j->out + j->ooff[i]);
    } else {
      zo_rx_packet_time((const zo_c16*)j->a + 64 * j->off[i], j->n[i], j->out + (size_t)i * j->stride, &j->res[i]);
    }
  }
  zo_vit_free(&v);
  return 0;
}
static int run_jobs(job_t* base, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  pthread_t th[256];
  job_t jobs[256];
  if (nthreads > 256) nthreads = 256;
  for (int t = 0; t < nthreads; t++) { jobs[t] = *base; jobs[t].t = t; jobs[t].nt = nthreads; }
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], 0, worker, &jobs[t]);
  worker(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], 0);
  return 0;
}
int zo_viterbi_batch(const int8_t* soft, const int64_t* soft_off, const int32_t* soft_len,
                     const int32_t* frame_len, const int16_t* code_rate, int npkts,
                     uint8_t* out, const int64_t* out_off, int nthreads) {
  job_t j; memset(&j, 0, sizeof(j));
  j.kind = 0; j.npkts = npkts; j.a = soft; j.off = soft_off; j.n = soft_len;
  j.fl = frame_len; j.cr = code_rate; j.out = out; j.ooff = out_off;
  return run_jobs(&j, nthreads);
}
int zo_rx_batch_time(const zo_c16* sym, const int64_t* sym_off, const int32_t* nsym, int npkts,
                     uint8_t* payload, int payload_stride, zo_rx_result* res, int nthreads) {
  job_t j; memset(&j, 0, sizeof(j));
  j.kind = 1; j.npkts = npkts; j.a = sym; j.off = sym_off; j.n = nsym;
  j.out = payload; j.stride = payload_stride; j.res = res;
  return run_jobs(&j, nthreads);
}

/* ------------------------------------------------------------------------------------ */
/* Synthetic TX, restating transmitter.blk:56-101 for workload generation in tests. */
/* encode12/23/34: code/WiFi/transmitter/encoding.blk:24-109 */
int zo_tx_encode(const uint8_t* bits, int nbits, int coding, uint8_t* coded) {
  int s = 0, k = 0;       /* s bit j = s[j] of the .blk */
  for (int i = 0; i < nbits; i++) {
    int b = bits[i] & 1;
    int A = b ^ bit_(s, 1) ^ bit_(s, 2) ^ bit_(s, 4) ^ bit_(s, 5);
    int B = b ^ bit_(s, 0) ^ bit_(s, 1) ^ bit_(s, 2) ^ bit_(s, 5);
    s = ((s << 1) | b) & 63;
    if (coding == 0) { coded[k++] = (uint8_t)A; coded[k++] = (uint8_t)B; }
    else if (coding == 2) {              /* encode34: A0 B0 | A1 | B2 */
      int ph = i % 3;
      if (ph == 0) { coded[k++] = (uint8_t)A; coded[k++] = (uint8_t)B; }
      else if (ph == 1) coded[k++] = (uint8_t)A;
      else coded[k++] = (uint8_t)B;
    } else {                             /* encode23: A0 B0 | A1 */
      int ph = i % 2;
      if (ph == 0) { coded[k++] = (uint8_t)A; coded[k++] = (uint8_t)B; }
      else coded[k++] = (uint8_t)A;
    }
  }
  return k;
}
/* modulating.blk (bpsk_mod_11a = 10720 and derived, const.blk:27-30) */
static void map_sym(int mod, const uint8_t* b, zo_c16* o) {
  const int16_t U1 = 10720, U2 = 7581, U4 = 3390, U6 = 1654;
  static const int g3[8] = {-7, -5, -1, -3, 7, 5, 1, 3};   /* index b0 b1 b2 (b0 MSB) */
  switch (mod) {
    case 0: o->re = b[0] ? U1 : -U1; o->im = 0; break;
    case 1: o->re = b[0] ? U2 : -U2; o->im = b[1] ? U2 : -U2; break;
    case 2: {
      static const int g2[4] = {-3, -1, 3, 1};             /* 00:-3 01:-1 10:3 11:1 */
      o->re = (int16_t)(g2[b[0] * 2 + b[1]] * U4); o->im = (int16_t)(g2[b[2] * 2 + b[3]] * U4); break;
    }
    default:
      o->re = (int16_t)(g3[b[0] * 4 + b[1] * 2 + b[2]] * U6);
      o->im = (int16_t)(g3[b[3] * 4 + b[4] * 2 + b[5]] * U6);
  }
}
static void interleave_map(int mod, const uint8_t* coded, zo_c16* sub48) {
  int N = zo_ncbps(mod), nb = N / 48;
  uint8_t il[288];
  for (int k = 0; k < N; k++) il[zo_deint_src(mod, k)] = coded[k];   /* interleaving.blk */
  for (int i = 0; i < 48; i++) map_sym(mod, il + nb * i, &sub48[i]);
}
int zo_tx_signal_symbol(int mod, int coding, int len, zo_c16* sub48) {
  /* createPLCPHeader: parsePLCPHeader.blk:47-116 */
  static const int rate[4][3] = {{0xB, -1, 0xF}, {0xA, -1, 0xE}, {0x9, -1, 0xD}, {-1, 0x8, 0xC}};
  int code = rate[mod][coding];
  if (code < 0) code = 0xB;
  uint8_t h[24] = {0};
  for (int k = 0; k < 4; k++) h[k] = (code >> k) & 1;
  for (int k = 0; k < 12; k++) h[5 + k] = (len >> k) & 1;
  int p = 0;
  for (int k = 0; k < 24; k++) p ^= h[k];
  h[17] ^= (uint8_t)p;
  uint8_t coded[48];
  zo_tx_encode(h, 24, 0, coded);
  interleave_map(0, coded, sub48);
  return 1;
}
/* SIGNAL symbol from the 24 header bits as given (emitHeader, parsePLCPHeader.blk:215-221):
   encode12 >>> interleaver_bpsk >>> modulate_bpsk */
int zo_tx_signal_from_bits(const uint8_t* hbits3, zo_c16* sub48) {
  uint8_t h[24], coded[48];
  for (int k = 0; k < 24; k++) h[k] = (hbits3[k >> 3] >> (k & 7)) & 1;
  zo_tx_encode(h, 24, 0, coded);
  interleave_map(0, coded, sub48);
  return 1;
}
/* tx_driver (transmitter.blk:56-101): crcXX(len,true) >>> scrambler(1011101) >>> encode >>>
   interleave >>> modulate.  Returns the number of data symbols. */
int zo_tx_data_symbols(const uint8_t* payload, int plen, int mod, int coding, zo_c16* sub48, int max_sym) {
  int nd = zo_ndbps(mod, coding), nc = zo_ncbps(mod);
  int so_far = 16 + plen * 8 + 32;
  int final_len = ((so_far + 6) + nd - 1) / nd * nd;
  int nsym = final_len / nd;
  if (nsym > max_sym) return -1;
  uint8_t* bits = (uint8_t*)calloc((size_t)final_len, 1);
  for (int k = 0; k < plen * 8; k++) bits[16 + k] = (payload[k >> 3] >> (k & 7)) & 1;
  uint32_t c = zo_crc32_bits(payload, plen);
  for (int k = 0; k < 32; k++) bits[16 + plen * 8 + k] = (c >> k) & 1;
  int st[7] = {1, 0, 1, 1, 1, 0, 1};
  for (int k = 0; k < final_len; k++) {
    int t = st[3] ^ st[0];
    for (int q = 0; q < 6; q++) st[q] = st[q + 1];
    st[6] = t;
    bits[k] ^= (uint8_t)t;
  }
  uint8_t* coded = (uint8_t*)malloc((size_t)nsym * nc);
  zo_tx_encode(bits, final_len, coding, coded);
  for (int s = 0; s < nsym; s++) interleave_map(mod, coded + (size_t)s * nc, sub48 + 48 * s);
  free(bits); free(coded);
  return nsym;
}
