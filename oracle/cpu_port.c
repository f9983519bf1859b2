/*
 * CPU PORT — test infrastructure only: the timed host-CPU baseline of bench.py (its
 * cpu_baseline leg, "kind": "port").  Not part of the product and never on the GPU path.
 *
 * The same receive chain as the oracle (zo_rx_batch_time: FFT >>> GetData >>> receiveBits,
 * code/WiFi/receiver/receiver.blk:43-54), written for speed on the host instead of for
 * side-by-side reading, and checked bit for bit against the oracle (tests/test_cpu_port.py):
 *   - FFT64 with precomputed twiddles (the oracle evaluates cos/sin per butterfly);
 *   - the Viterbi brick loop (csrc/sora_ext_viterbi.cpp:66-153) with the 64-state ACS of
 *     viterbicore.hpp:105-147 on one AVX-512 register (vpermb gathers the two predecessor
 *     metrics and the branch metrics, u8 wrapping adds, min_epu8, the survivor word from the
 *     metric LSBs), scalar traceback;
 *   - descrambler by bytes from a 7-bit state table and CRC-32 by a byte table (crc.blk's
 *     generic update is the reflected CRC-32 of zlib: tests/test_oracle_golden.py).
 * Packet-parallel over pthreads.  Without AVX-512 (VBMI) on the host the Viterbi falls
 * back to the oracle's scalar brick loop.
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "ziria_oracle.h"

/* ---------------------------------------------------------------- FFT64 with tables */
static zo_c16 g_tw64[3][16], g_tw16[3][4];
/* the same twiddles as madd operand pairs, 16 complex per row: [k][0] = (re, ~im) gives the
   real part of mul_shiftx, [k][1] = (im, re) the imaginary part; stage-16 rows repeat 4x */
static uint32_t g_w64[3][2][16] __attribute__((aligned(64))), g_w16[3][2][16] __attribute__((aligned(64)));
static uint32_t g_crc_tab[256];
static uint8_t g_scr_byte[128], g_scr_next[128];       /* descrambler: 8 steps from a 7-bit state */
static uint16_t g_deint[4][288];                       /* deinterleaver source index by modulation */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void init_tables(void) {
  for (int k = 1; k <= 3; k++) {
    for (int n = 0; n < 16; n++) zo_twiddle(64, k, n, &g_tw64[k - 1][n].re, &g_tw64[k - 1][n].im);
    for (int n = 0; n < 4; n++) zo_twiddle(16, k, n, &g_tw16[k - 1][n].re, &g_tw16[k - 1][n].im);
    for (int n = 0; n < 16; n++) {
      const zo_c16 a = g_tw64[k - 1][n], b = g_tw16[k - 1][n & 3];
      g_w64[k - 1][0][n] = (uint16_t)a.re | (uint32_t)(uint16_t)~a.im << 16;
      g_w64[k - 1][1][n] = (uint16_t)a.im | (uint32_t)(uint16_t)a.re << 16;
      g_w16[k - 1][0][n] = (uint16_t)b.re | (uint32_t)(uint16_t)~b.im << 16;
      g_w16[k - 1][1][n] = (uint16_t)b.im | (uint32_t)(uint16_t)b.re << 16;
    }
  }
  for (int mod = 0; mod < 4; mod++)
    for (int k = 0; k < zo_ncbps(mod); k++) g_deint[mod][k] = (uint16_t)zo_deint_src(mod, k);
  for (uint32_t b = 0; b < 256; b++) {
    uint32_t c = b;
    for (int j = 0; j < 8; j++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    g_crc_tab[b] = c;
  }
  /* scramble.blk:28-44 on a state st[0..6] (st bit q = state bit q): t = st3 ^ st0, shift
     down, st6 = t; the keystream bit is t */
  for (int s = 0; s < 128; s++) {
    int st = s, byte = 0;
    for (int j = 0; j < 8; j++) {
      const int t = ((st >> 3) ^ st) & 1;
      st = (st >> 1) | (t << 6);
      byte |= t << j;
    }
    g_scr_byte[s] = (uint8_t)byte;
    g_scr_next[s] = (uint8_t)st;
  }
}

static inline int16_t sat16(int32_t x) { return (int16_t)(x > 32767 ? 32767 : (x < -32768 ? -32768 : x)); }
static inline zo_c16 cadd(zo_c16 a, zo_c16 b) { zo_c16 r = {sat16(a.re + b.re), sat16(a.im + b.im)}; return r; }
static inline zo_c16 csub(zo_c16 a, zo_c16 b) { zo_c16 r = {sat16(a.re - b.re), sat16(a.im - b.im)}; return r; }
static inline zo_c16 shr2(zo_c16 a) { zo_c16 r = {(int16_t)(a.re >> 2), (int16_t)(a.im >> 2)}; return r; }
static inline zo_c16 mulw(zo_c16 a, zo_c16 w) {          /* mul_shiftx: madd wrap, >> 15, low 16 */
  const int32_t re = (int32_t)((uint32_t)(a.re * w.re) + (uint32_t)(a.im * (int16_t)~w.im));
  const int32_t im = (int32_t)((uint32_t)(a.re * w.im) + (uint32_t)(a.im * w.re));
  zo_c16 r = {(int16_t)(re >> 15), (int16_t)(im >> 15)};
  return r;
}
static inline void stage(zo_c16* x, int N, const zo_c16* tw1, const zo_c16* tw2, const zo_c16* tw3) {
  const int q = N / 4;
  for (int n = 0; n < q; n++) {
    const zo_c16 a = shr2(x[n]), b = shr2(x[n + q]), c = shr2(x[n + 2 * q]), d = shr2(x[n + 3 * q]);
    const zo_c16 ac = cadd(a, c), bd = cadd(b, d), a_c = csub(a, c), b_d = csub(b, d);
    const zo_c16 jb = {(int16_t)~b_d.im, b_d.re};
    x[n] = cadd(ac, bd);
    x[n + q] = mulw(csub(ac, bd), tw2[n]);
    x[n + 2 * q] = mulw(csub(a_c, jb), tw1[n]);
    x[n + 3 * q] = mulw(cadd(a_c, jb), tw3[n]);
  }
}
static inline void fft4(zo_c16* x) {
  const zo_c16 y0 = shr2(x[0]), y1 = shr2(x[1]), y2 = shr2(x[2]), y3 = shr2(x[3]);
  const zo_c16 A = cadd(y0, y2), B = cadd(y1, y3);
  const zo_c16 L = {sat16(y0.re + (int16_t)~y2.re), sat16(y0.im + (int16_t)~y2.im)};
  const zo_c16 T = {sat16(y1.re + (int16_t)~y3.re), sat16(y1.im + (int16_t)~y3.im)};
  const zo_c16 jT = {(int16_t)~T.im, T.re}, njT = {(int16_t)~jT.re, (int16_t)~jT.im};
  const zo_c16 nB = {(int16_t)~B.re, (int16_t)~B.im};
  x[0] = cadd(A, B);
  x[1] = cadd(nB, A);
  x[2] = cadd(L, njT);
  x[3] = cadd(L, jT);
}
static void fft64_fast(const zo_c16* in, zo_c16* out) {
  zo_c16 x[64];
  memcpy(x, in, sizeof(x));
  stage(x, 64, g_tw64[0], g_tw64[1], g_tw64[2]);
  for (int q = 0; q < 4; q++) {
    stage(x + 16 * q, 16, g_tw16[0], g_tw16[1], g_tw16[2]);
    for (int r = 0; r < 4; r++) fft4(x + 16 * q + 4 * r);
  }
  for (int i = 0; i < 64; i++) {
    const int b = ((i & 1) << 5) | ((i & 2) << 3) | ((i & 4) << 1) | ((i & 8) >> 1) | ((i & 16) >> 3) | ((i & 32) >> 5);
    out[i] = x[b];
  }
}

/* The same FFT64 on AVX-512, 16 complex16 values per register (the reference's FFTSSE
   bricks hold 4 per SSE register): saturating adds, madd-wrap mul_shiftx, XOR-as-negate, so
   the result is fft64_fast's bit for bit.  Stage 64 runs on x[0..15] .. x[48..63] as they
   lie; a 128-bit-lane transpose puts the four 16-point sub-blocks side by side for stage 16;
   a 32-bit transpose within lanes lines up the 4-point base cases; one permute per output
   block undoes the bit reversal. */
#define AVX512_FFT __attribute__((target("avx512f,avx512bw,avx512vbmi")))
AVX512_FFT static inline __m512i v_not(__m512i x) { return _mm512_xor_si512(x, _mm512_set1_epi32(-1)); }
AVX512_FFT static inline __m512i v_mulj(__m512i x) {      /* (re, im) -> (~im, re) */
  return _mm512_xor_si512(_mm512_rol_epi32(x, 16), _mm512_set1_epi32(0xFFFF));
}
AVX512_FFT static inline __m512i v_mulw(__m512i a, const uint32_t* w) {
  const __m512i re = _mm512_madd_epi16(a, _mm512_load_si512(w)), im = _mm512_madd_epi16(a, _mm512_load_si512(w + 16));
  return _mm512_mask_blend_epi16(0xAAAAAAAAu, _mm512_srli_epi32(re, 15), _mm512_slli_epi32(im, 1));
}
AVX512_FFT static inline void v_stage(__m512i* a, __m512i* b, __m512i* c, __m512i* d, const uint32_t (*w)[2][16]) {
  const __m512i A = _mm512_srai_epi16(*a, 2), B = _mm512_srai_epi16(*b, 2), C = _mm512_srai_epi16(*c, 2),
                D = _mm512_srai_epi16(*d, 2);
  const __m512i ac = _mm512_adds_epi16(A, C), bd = _mm512_adds_epi16(B, D), a_c = _mm512_subs_epi16(A, C),
                jb = v_mulj(_mm512_subs_epi16(B, D));
  *a = _mm512_adds_epi16(ac, bd);
  *b = v_mulw(_mm512_subs_epi16(ac, bd), w[1][0]);
  *c = v_mulw(_mm512_subs_epi16(a_c, jb), w[0][0]);
  *d = v_mulw(_mm512_adds_epi16(a_c, jb), w[2][0]);
}
AVX512_FFT static void fft64_avx512(const zo_c16* in, zo_c16* out) {
  __m512i y0 = _mm512_loadu_si512(in), y1 = _mm512_loadu_si512(in + 16), y2 = _mm512_loadu_si512(in + 32),
          y3 = _mm512_loadu_si512(in + 48);
  v_stage(&y0, &y1, &y2, &y3, g_w64);                   /* y_k = sub-block k (x[16k .. 16k+15]) */
  const __m512i t0 = _mm512_shuffle_i64x2(y0, y1, 0x44), t1 = _mm512_shuffle_i64x2(y0, y1, 0xEE),
                t2 = _mm512_shuffle_i64x2(y2, y3, 0x44), t3 = _mm512_shuffle_i64x2(y2, y3, 0xEE);
  __m512i v0 = _mm512_shuffle_i64x2(t0, t2, 0x88), v1 = _mm512_shuffle_i64x2(t0, t2, 0xDD),
          v2 = _mm512_shuffle_i64x2(t1, t3, 0x88), v3 = _mm512_shuffle_i64x2(t1, t3, 0xDD);
  v_stage(&v0, &v1, &v2, &v3, g_w16);                   /* v_r lane k = x[16k + 4r .. 16k + 4r + 3] */
  const __m512i u0 = _mm512_unpacklo_epi32(v0, v1), u1 = _mm512_unpackhi_epi32(v0, v1),
                u2 = _mm512_unpacklo_epi32(v2, v3), u3 = _mm512_unpackhi_epi32(v2, v3);
  const __m512i e0 = _mm512_srai_epi16(_mm512_unpacklo_epi64(u0, u2), 2),
                e1 = _mm512_srai_epi16(_mm512_unpackhi_epi64(u0, u2), 2),
                e2 = _mm512_srai_epi16(_mm512_unpacklo_epi64(u1, u3), 2),
                e3 = _mm512_srai_epi16(_mm512_unpackhi_epi64(u1, u3), 2);   /* e_i[4k + r] = x[16k + 4r + i] */
  const __m512i A = _mm512_adds_epi16(e0, e2), B = _mm512_adds_epi16(e1, e3);  /* FFTSSEEx<4>, as fft4 */
  const __m512i L = _mm512_adds_epi16(e0, v_not(e2)), T = _mm512_adds_epi16(e1, v_not(e3));
  const __m512i jT = v_mulj(T);
  const __m512i f[4] = {_mm512_adds_epi16(A, B), _mm512_adds_epi16(v_not(B), A), _mm512_adds_epi16(L, v_not(jT)),
                        _mm512_adds_epi16(L, jT)};
  /* out[k] = x[bitrev6(k)]: block k >> 4 = 2 k5 + k4 comes from f[2 k4 + k5], element bitrev4(k & 15) */
  const __m512i rev4 = _mm512_setr_epi32(0, 8, 4, 12, 2, 10, 6, 14, 1, 9, 5, 13, 3, 11, 7, 15);
  _mm512_storeu_si512(out, _mm512_permutexvar_epi32(rev4, f[0]));
  _mm512_storeu_si512(out + 16, _mm512_permutexvar_epi32(rev4, f[2]));
  _mm512_storeu_si512(out + 32, _mm512_permutexvar_epi32(rev4, f[1]));
  _mm512_storeu_si512(out + 48, _mm512_permutexvar_epi32(rev4, f[3]));
}

/* GetData (GetData.blk:24-35) >>> DemapLimit >>> Demap >>> Deinterleave of one FFT output,
   as zo_get_data / zo_demap_limit / zo_demap / zo_deinterleave with the permutation in a table */
static void symbol_soft(const zo_c16* f, int mod, int8_t* di) {
  static const int seg[6][2] = {{38, 5}, {44, 13}, {58, 6}, {1, 6}, {8, 13}, {22, 5}};
  const uint8_t *B = zo_lut(0), *Q16 = zo_lut(1), *Q2 = zo_lut(2), *Q3 = zo_lut(3);
  int8_t soft[288];
  int k = 0;
  for (int g = 0; g < 6; g++)
    for (int i = 0; i < seg[g][1]; i++) {
      const zo_c16 v = f[seg[g][0] + i];
      const int re = (v.re < -128 ? -128 : v.re > 127 ? 127 : v.re) & 0xFF;
      const int im = (v.im < -128 ? -128 : v.im > 127 ? 127 : v.im) & 0xFF;
      switch (mod) {
        case 0: soft[k++] = (int8_t)B[re]; break;
        case 1: soft[k++] = (int8_t)B[re]; soft[k++] = (int8_t)B[im]; break;
        case 2: soft[k++] = (int8_t)B[re]; soft[k++] = (int8_t)Q16[re];
                soft[k++] = (int8_t)B[im]; soft[k++] = (int8_t)Q16[im]; break;
        default: soft[k++] = (int8_t)B[re]; soft[k++] = (int8_t)Q2[re]; soft[k++] = (int8_t)Q3[re];
                 soft[k++] = (int8_t)B[im]; soft[k++] = (int8_t)Q2[im]; soft[k++] = (int8_t)Q3[im];
      }
    }
  const uint16_t* P = g_deint[mod];
  for (int j = 0; j < k; j++) di[j] = soft[P[j]];
}

/* ---------------------------------------------------------------- Viterbi, AVX-512 ACS */
typedef struct {
  uint8_t m[64];
  uint64_t* surv;
  uint32_t cap, tr, ob, frame_len, cr;
} pv_t;

static inline int bit_(int v, int b) { return (v >> b) & 1; }
static uint8_t g_idx0[64], g_idx1[64], g_p0[64], g_p1[64];
static void init_vit_tables(void) {
  for (int s = 0; s < 64; s++) {
    const int p0 = s >> 1, p1 = p0 | 32, x = s & 1;
    const int a0 = x ^ bit_(p0, 1) ^ bit_(p0, 2) ^ bit_(p0, 4) ^ bit_(p0, 5), b0 = x ^ bit_(p0, 0) ^ bit_(p0, 1) ^ bit_(p0, 2) ^ bit_(p0, 5);
    const int a1 = x ^ bit_(p1, 1) ^ bit_(p1, 2) ^ bit_(p1, 4) ^ bit_(p1, 5), b1 = x ^ bit_(p1, 0) ^ bit_(p1, 1) ^ bit_(p1, 2) ^ bit_(p1, 5);
    g_idx0[s] = (uint8_t)(2 * a0 + b0);
    g_idx1[s] = (uint8_t)(2 * a1 + b1);
    g_p0[s] = (uint8_t)p0;
    g_p1[s] = (uint8_t)p1;
  }
}

/* traceback: csrc/viterbicore.hpp:170-239 (as the oracle) */
static void pv_traceback(const uint8_t* m, const uint64_t* surv, uint32_t col, uint8_t* out, uint32_t nbits,
                         uint32_t look) {
  int best = 0x7FFFFFFF;
  for (int s = 0; s < 64; s++) {
    const int key = (int16_t)(uint16_t)((m[s] << 8) | (4 * s));
    if (key < best) best = key;
  }
  int i = (best >> 2) & 0x7F;
  uint32_t t = col;
  for (uint32_t k = 0; k < look; k++) {
    t--;
    i = ((i >> 1) & 0x3F) | (int)((surv[t] >> ((i >> 1) & 0x3F)) & 1) << 6;
  }
  for (uint32_t byte = nbits >> 3; byte-- > 0;) {
    int oc = 0;
    for (int j = 0; j < 8; j++) {
      oc = (oc << 1) | ((i >> 6) & 1);
      t--;
      i = ((i >> 1) & 0x3F) | (int)((surv[t] >> ((i >> 1) & 0x3F)) & 1) << 6;
    }
    out[byte] = (uint8_t)oc;
  }
}

__attribute__((target("avx512f,avx512bw,avx512vbmi")))
static int pv_decode_avx512(pv_t* v, const int8_t* soft, int n, uint8_t* out) {
  const __m512i idx0 = _mm512_loadu_si512(g_idx0), idx1 = _mm512_loadu_si512(g_idx1);
  const __m512i pp0 = _mm512_loadu_si512(g_p0), pp1 = _mm512_loadu_si512(g_p1);
  const __m512i fe = _mm512_set1_epi8((char)0xFE), one = _mm512_set1_epi8(1);
  __m512i m = _mm512_loadu_si512(v->m);
  const uint8_t* in = (const uint8_t*)soft;
  const int G = v->cr == 0 ? 2 : v->cr == 1 ? 3 : 4;
  uint32_t total = 0;
  const uint32_t tr_end = v->frame_len * 8 + 6;
  for (int g = 0; g + G <= n; g += G) {
    const int ns = v->cr + 1;
    if (v->tr + (uint32_t)ns >= 40000u) break;        /* TRELLIS_MAX (sora_ext_viterbi.cpp:39): as zo_vit_decode */
    for (int st = 0; st < ns; st++) {
      int t0, t1, t2, t3;                              /* BM table by 2A+B: BM(v,e) = e ? 14-2v : 2v */
      if (st == 0) {
        const int a = in[g], b = in[g + 1];
        t0 = 2 * a + 2 * b; t1 = 2 * a + 14 - 2 * b; t2 = 14 - 2 * a + 2 * b; t3 = 28 - 2 * a - 2 * b;
      } else if (st == 1) {                            /* A only */
        const int a = in[g + 2];
        t0 = t1 = 2 * a; t2 = t3 = 14 - 2 * a;
      } else {                                         /* B only */
        const int a = in[g + 3];
        t0 = t2 = 2 * a; t1 = t3 = 14 - 2 * a;
      }
      const __m512i T = _mm512_set1_epi32((int)((uint32_t)t0 | ((uint32_t)t1 << 8) | ((uint32_t)t2 << 16) | ((uint32_t)t3 << 24)));
      const __m512i bm0 = _mm512_permutexvar_epi8(idx0, T), bm1 = _mm512_permutexvar_epi8(idx1, T);
      const __m512i r0 = _mm512_and_si512(_mm512_add_epi8(_mm512_permutexvar_epi8(pp0, m), bm0), fe);
      const __m512i r1 = _mm512_or_si512(_mm512_add_epi8(_mm512_permutexvar_epi8(pp1, m), bm1), one);
      m = _mm512_min_epu8(r0, r1);
      v->tr++;
      if (v->tr < v->cap) v->surv[v->tr] = _mm512_test_epi8_mask(m, one);
    }
    const uint32_t tr = v->tr;
    if ((tr & 7) == 0) {                               /* normalize: csrc/viterbicore.hpp:149-168 */
      __m512i t = _mm512_min_epu8(m, _mm512_shuffle_i64x2(m, m, 0x4E));          /* 256-bit halves */
      t = _mm512_min_epu8(t, _mm512_shuffle_i64x2(t, t, 0xB1));                   /* 128-bit */
      t = _mm512_min_epu8(t, _mm512_shuffle_epi32(t, (_MM_PERM_ENUM)0x4E));       /* 64-bit */
      t = _mm512_min_epu8(t, _mm512_shuffle_epi32(t, (_MM_PERM_ENUM)0xB1));       /* 32-bit */
      t = _mm512_min_epu8(t, _mm512_srli_epi32(t, 16));
      t = _mm512_min_epu8(t, _mm512_srli_epi32(t, 8));                            /* byte 0: the min */
      const __m512i mn = _mm512_and_si512(_mm512_permutexvar_epi8(_mm512_setzero_si512(), t), fe);
      m = _mm512_sub_epi8(m, mn);
    }
    uint32_t cnt = 0, look = 0;
    if (tr >= tr_end) { cnt = tr_end - v->ob - 6; look = tr - tr_end; }
    else if (tr >= v->ob + 286) { cnt = 256; look = 24 + ((tr - (v->ob + 286)) & 7); }
    if (cnt) {
      uint8_t mm[64];
      _mm512_storeu_si512(mm, m);
      pv_traceback(mm, v->surv, tr, out + total / 8, cnt, look);
      v->ob += cnt;
      total += cnt;
    }
  }
  _mm512_storeu_si512(v->m, m);
  return (int)total;
}

/* ---------------------------------------------------------------- descramble + CRC */
static int descramble_crc_fast(const uint8_t* dec, int len, uint8_t* payload) {
  int st = 0;
  for (int k = 0; k < 7; k++) st |= ((dec[(9 + k) >> 3] >> ((9 + k) & 7)) & 1) << k;
  uint8_t* tmp = (uint8_t*)malloc((size_t)len + 8);
  for (int b = 0; b < len; b++) {                      /* bits 16 + 8b .. : byte b + 2 of dec */
    tmp[b] = (uint8_t)(dec[b + 2] ^ g_scr_byte[st]);
    st = g_scr_next[st];
  }
  const int plen = len >= 4 ? len - 4 : 0;
  memcpy(payload, tmp, (size_t)plen);
  uint32_t c = 0xFFFFFFFFu;
  for (int b = 0; b < plen; b++) c = (c >> 8) ^ g_crc_tab[(c ^ tmp[b]) & 0xFFu];
  c = ~c;
  const uint32_t rx = (uint32_t)tmp[plen] | ((uint32_t)tmp[plen + 1] << 8) | ((uint32_t)tmp[plen + 2] << 16) |
                      ((uint32_t)tmp[plen + 3] << 24);
  free(tmp);
  return len >= 4 && c == rx;
}

/* ---------------------------------------------------------------- one packet */
static int have_avx512(void) {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("avx512vbmi");
}
static int g_avx;

/* FFT of symbol k of a packet; with chan64 (the EQ chain, receiver.blk:66-69) followed by
   ChannelEqualization and PilotTrack (the oracle's restatements, ziria_oracle_eq.c) */
static inline void fft_sym(const zo_c16* in, int k, const zo_c16* chan64, zo_c16* f) {
  if (!chan64) {
    if (g_avx) fft64_avx512(in, f); else fft64_fast(in, f);
    return;
  }
  zo_c16 t[64], e[64];
  if (g_avx) fft64_avx512(in, t); else fft64_fast(in, t);
  zo_channel_eq(t, chan64, e);
  zo_pilot_track(e, k, f);
}

static void rx_packet(const zo_c16* sym, int nsym, const zo_c16* chan64, uint8_t* payload, zo_rx_result* r, pv_t* v,
                      zo_vit* zv) {
  memset(r, 0, sizeof(*r));
  if (nsym < 1) return;
  zo_c16 f[64], sub[48], lim[48];
  int8_t soft[288], di[288];
  fft_sym(sym, 0, chan64, f);                          /* SIGNAL: DecodePLCP.blk:30-37 */
  zo_get_data(f, sub);
  zo_demap_limit(sub, 48, lim);
  zo_demap(0, lim, soft);
  zo_deinterleave(0, soft, di);
  uint8_t hb[4] = {0, 0, 0, 0};
  zo_vit_sig(di, hb);
  hb[2] &= 0x03;
  hb[3] = 0;
  zo_parse_header(hb, &r->h);
  const int mod = r->h.modulation, cod = r->h.coding, len = r->h.len, nc = zo_ncbps(mod);
  uint8_t* dec = (uint8_t*)calloc((size_t)len + 16, 1);
  int bits = 0, used = 0;
  if (g_avx) {
    for (int s = 0; s < 64; s++) v->m[s] = s ? 48 : 0;  /* ALL_INIT0 */
    v->tr = v->ob = 0; v->frame_len = (uint32_t)len + 2; v->cr = (uint32_t)cod;
    v->surv[0] = 0;
  } else {
    zo_vit_init(zv, len + 2, cod, 256);
  }
  for (int k = 0; k < nsym - 1 && bits < (len + 2) * 8; k++) {
    fft_sym(sym + 64 * (1 + k), 1 + k, chan64, f);
    symbol_soft(f, mod, di);
    for (int c = 0; c < nc; c += 48)
      bits += g_avx ? pv_decode_avx512(v, di + c, 48, dec + bits / 8) : zo_vit_decode(zv, di + c, 48, dec + bits / 8);
    used++;
  }
  r->nsym_used = 1 + used;
  r->viterbi_bits = bits;
  r->crc_ok = bits >= (len + 2) * 8 ? descramble_crc_fast(dec, len, payload) : 0;
  free(dec);
}

typedef struct {
  const zo_c16* sym; const int64_t* off; const int32_t* n;
  uint8_t* out; int stride; zo_rx_result* res; int npkts;
  int* next;                                           /* shared packet counter (dynamic claim) */
  const zo_c16* chan;                                  /* EQ chain: 64 coefficients per packet, else null */
} pjob_t;
static void* pworker(void* p) {
  pjob_t* j = (pjob_t*)p;
  pv_t v; memset(&v, 0, sizeof(v));
  v.cap = 40000 + 8;
  v.surv = (uint64_t*)calloc(v.cap, sizeof(uint64_t));
  zo_vit zv; memset(&zv, 0, sizeof(zv));
  for (int i; (i = __atomic_fetch_add(j->next, 1, __ATOMIC_RELAXED)) < j->npkts;)
    rx_packet(j->sym + 64 * j->off[i], j->n[i], j->chan ? j->chan + 64 * (size_t)i : 0, j->out + (size_t)i * j->stride,
              &j->res[i], &v, &zv);
  free(v.surv);
  zo_vit_free(&zv);
  return 0;
}
static void init_all(void) { init_tables(); init_vit_tables(); g_avx = have_avx512(); }

/* Same contract as zo_viterbi_batch (init + decode of all soft values per packet, depth
   256), packet-parallel with dynamic claiming. */
typedef struct {
  const int8_t* soft; const int64_t* soft_off; const int32_t* soft_len; const int32_t* frame_len;
  const int16_t* code_rate; uint8_t* out; const int64_t* out_off; int npkts; int* next;
} vjob_t;
static void* vworker(void* p) {
  vjob_t* j = (vjob_t*)p;
  pv_t v; memset(&v, 0, sizeof(v));
  v.cap = 40000 + 8;
  v.surv = (uint64_t*)calloc(v.cap, sizeof(uint64_t));
  zo_vit zv; memset(&zv, 0, sizeof(zv));
  for (int i; (i = __atomic_fetch_add(j->next, 1, __ATOMIC_RELAXED)) < j->npkts;) {
    const int8_t* s = j->soft + j->soft_off[i];
    uint8_t* o = j->out + j->out_off[i];
    if (g_avx) {
      for (int q = 0; q < 64; q++) v.m[q] = q ? 48 : 0;
      v.tr = v.ob = 0; v.frame_len = (uint32_t)j->frame_len[i]; v.cr = (uint32_t)j->code_rate[i];
      v.surv[0] = 0;
      pv_decode_avx512(&v, s, j->soft_len[i], o);
    } else {
      zo_vit_init(&zv, j->frame_len[i], j->code_rate[i], 256);
      zo_vit_decode(&zv, s, j->soft_len[i], o);
    }
  }
  free(v.surv);
  zo_vit_free(&zv);
  return 0;
}
int zp_viterbi_batch(const int8_t* soft, const int64_t* soft_off, const int32_t* soft_len,
                     const int32_t* frame_len, const int16_t* code_rate, int npkts,
                     uint8_t* out, const int64_t* out_off, int nthreads) {
  pthread_once(&g_once, init_all);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  int next = 0;
  vjob_t j = {soft, soft_off, soft_len, frame_len, code_rate, out, out_off, npkts, &next};
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], 0, vworker, &j);
  vworker(&j);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], 0);
  return g_avx;
}

/* n FFT64s by the port's own FFT (tests/test_cpu_port.py compares them with the oracle's) */
int zp_fft64(const zo_c16* in, zo_c16* out, int n) {
  pthread_once(&g_once, init_all);
  for (int i = 0; i < n; i++) {
    if (g_avx) fft64_avx512(in + 64 * i, out + 64 * i); else fft64_fast(in + 64 * i, out + 64 * i);
  }
  return g_avx;
}

static int rx_batch(const zo_c16* sym, const int64_t* sym_off, const int32_t* nsym, int npkts, const zo_c16* chan,
                    uint8_t* payload, int payload_stride, zo_rx_result* res, int nthreads) {
  pthread_once(&g_once, init_all);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  pjob_t jobs[256];
  int next = 0;
  for (int t = 0; t < nthreads; t++) {
    pjob_t j = {sym, sym_off, nsym, payload, payload_stride, res, npkts, &next, chan};
    jobs[t] = j;
  }
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], 0, pworker, &jobs[t]);
  pworker(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], 0);
  return g_avx;
}

/* Same contract as zo_rx_batch_time.  Returns 1 when the AVX-512 ACS ran, 0 otherwise. */
int zp_rx_batch_time(const zo_c16* sym, const int64_t* sym_off, const int32_t* nsym, int npkts,
                     uint8_t* payload, int payload_stride, zo_rx_result* res, int nthreads) {
  return rx_batch(sym, sym_off, nsym, npkts, 0, payload, payload_stride, res, nthreads);
}
/* Same contract as zo_rx_batch_time_eq (FFT >>> ChannelEqualization >>> PilotTrack >>> ...). */
int zp_rx_batch_time_eq(const zo_c16* sym, const int64_t* sym_off, const int32_t* nsym, int npkts, const zo_c16* chan,
                        uint8_t* payload, int payload_stride, zo_rx_result* res, int nthreads) {
  return rx_batch(sym, sym_off, nsym, npkts, chan, payload, payload_stride, res, nthreads);
}
