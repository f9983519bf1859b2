// Per-call externals of libziria_rx.so on the host CPU ("the exact
// symbols ... with identical per-call semantics: a CPU path, with the GPU used only if
// batched").  A wplc-generated receiver calls __ext_sora_fft once per OFDM symbol and
// __ext_viterbi_brick_decode_fast once per 48 soft values and needs the answer before the
// next call, so a GPU launch + sync per call (10-65 us) cannot compete with a host core; the
// batched externals (zrx_api.hip) are where the GPU decodes.
//
// The SIMD functions carry __attribute__((target("avx2"))); the file is compiled without
// -mavx2, so nothing else (static initializers, the plan code) uses AVX2 and require_avx2()
// can report a host without it before any AVX2 instruction runs.
//   FFT      FFTSafe<N> (csrc/fft_r4difx.hpp:220-237, csrc/sora_ext_lib.cpp:2672-2812) for every
//            size, executing the plans of zrx_fftplan.hpp with the SSE bricks' integer
//            semantics; FFT64 (the WiFi symbol) has a dedicated AVX2 path.
//   Viterbi  the brick (csrc/sora_ext_viterbi.cpp:38-194, csrc/viterbicore.hpp:57-399): the 64
//            u8 metrics live in two ymm registers (states 0..31, 32..63); one trellis column
//            is 2 byte shuffles (branch metrics), 4 adds, AND/OR markers, 2 min_epu8 and an
//            interleave; the survivor markers are kept as one 64-bit word per column
//            (movemask), the traceback walks those words.
#include <immintrin.h>
#include <stdint.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define ZRX_C_LINKAGE_EXTERNALS
#include "../../include/ziria_rx.h"
#include "zrx_fftplan.hpp"
#include "zrx_internal.h"

namespace {

void require_avx2() {
  static const bool ok = __builtin_cpu_supports("avx2");
  if (!ok) {
    std::fprintf(stderr, "ziria_rx: the per-call externals need an AVX2 host CPU\n");
    std::abort();
  }
}

// ------------------------------------------------------------------ FFT (any size, plans)
struct c16 { int16_t re, im; };
inline int16_t sat16(int32_t x) { return (int16_t)(x > 32767 ? 32767 : (x < -32768 ? -32768 : x)); }
inline c16 sadd(c16 a, c16 b) { return {sat16(a.re + b.re), sat16(a.im + b.im)}; }     // adds_epi16
inline c16 ssub(c16 a, c16 b) { return {sat16(a.re - b.re), sat16(a.im - b.im)}; }     // subs_epi16
inline c16 sra(c16 a, int s) { return {(int16_t)(a.re >> s), (int16_t)(a.im >> s)}; }  // srai_epi16
inline c16 inv(c16 a) { return {(int16_t)~a.re, (int16_t)~a.im}; }                     // XOR-as-negate
inline c16 mulj(c16 a) { return {(int16_t)~a.im, a.re}; }                              // mul_jx
// mul_shiftx(a, b, 15) (csrc/sora_ext_lib_fft.hpp:42-67): madd_epi16 on (re, ~im) / (im, re),
// 32-bit wrapping sum of two exact products, srai 15, low 16 bits
inline c16 mul_shift(c16 a, int16_t bre, int16_t bim) {
  const int32_t re = (int32_t)((uint32_t)(a.re * bre) + (uint32_t)(a.im * (int16_t)~bim));
  const int32_t im = (int32_t)((uint32_t)(a.re * bim) + (uint32_t)(a.im * bre));
  return {(int16_t)(re >> 15), (int16_t)(im >> 15)};
}
inline c16 mul_tw(c16 a, uint32_t t) { return mul_shift(a, (int16_t)(t & 0xFFFF), (int16_t)(t >> 16)); }

// FFTSSEEx<4> (csrc/fft_r4difx.hpp:111-140) regrouped on (re, im) pairs
void fft4(c16* x) {
  const c16 y0 = sra(x[0], 2), y1 = sra(x[1], 2), y2 = sra(x[2], 2), y3 = sra(x[3], 2);
  const c16 A = sadd(y0, y2), B = sadd(y1, y3), L = sadd(y0, inv(y2)), T = sadd(y1, inv(y3));
  const c16 jT = mulj(T);
  x[0] = sadd(A, B);
  x[1] = sadd(inv(B), A);
  x[2] = sadd(L, inv(jT));
  x[3] = sadd(L, jT);
}
// FFTSSEEx<8> (csrc/fft_r4difx.hpp:142-218)
void fft8(c16* x) {
  c16 d[4], s[4];
  for (int k = 0; k < 4; k++) {
    const c16 a = sra(x[k], 3), b = sra(x[k + 4], 3);
    d[k] = ssub(a, b);
    s[k] = sadd(a, b);
  }
  const c16 m2 = {d[2].im, (int16_t)~d[2].re}, m3 = {d[3].im, (int16_t)~d[3].re};
  const c16 f0 = mul_shift(sadd(d[0], m2), 32767, 0), f1 = mul_shift(sadd(d[1], m3), 23169, -23169);
  const c16 f2 = mul_shift(sadd(inv(m2), d[0]), 32767, 0), f3 = mul_shift(sadd(inv(m3), d[1]), -23169, -23169);
  const c16 t0 = sadd(s[0], s[2]), t1 = sadd(s[1], s[3]), t2 = sadd(inv(s[2]), s[0]);
  const c16 t3a = sadd(inv(s[3]), s[1]);
  const c16 t3 = {t3a.im, (int16_t)~t3a.re};
  x[0] = sadd(t0, t1);
  x[1] = sadd(inv(t1), t0);
  x[2] = sadd(t2, t3);
  x[3] = sadd(inv(t3), t2);
  x[4] = sadd(f0, f1);
  x[5] = sadd(f0, inv(f1));
  x[6] = sadd(f2, f3);
  x[7] = sadd(f2, inv(f3));
}
// One DIF butterfly of radix r over x[base + q m] (FFTSSE<M> csrc/fft_r4difx.hpp:54-97,
// FFTSSE_3<M> csrc/sora_ext_lib_fft.hpp:111-171, FFTSSE_5<M> :253-349)
void butterfly(c16* x, int radix, int base, int m, int n, const uint32_t* tw) {
  if (radix == 4) {
    const c16 a = sra(x[base], 2), b = sra(x[base + m], 2), c = sra(x[base + 2 * m], 2), d = sra(x[base + 3 * m], 2);
    const c16 ac = sadd(a, c), bd = sadd(b, d), a_c = ssub(a, c), b_d = ssub(b, d);
    const c16 jb = mulj(b_d);
    x[base] = sadd(ac, bd);
    x[base + m] = mul_tw(ssub(ac, bd), tw[m + n]);
    x[base + 2 * m] = mul_tw(ssub(a_c, jb), tw[n]);
    x[base + 3 * m] = mul_tw(sadd(a_c, jb), tw[2 * m + n]);
  } else if (radix == 3) {
    const c16 a = sra(x[base], 2), b = sra(x[base + m], 2), c = sra(x[base + 2 * m], 2);
    const c16 bk1 = mul_shift(b, -16384, -28378), bk2 = mul_shift(b, -16384, 28378);
    const c16 ck1 = mul_shift(c, -16384, -28378), ck2 = mul_shift(c, -16384, 28378);
    x[base] = sadd(sadd(a, b), c);
    x[base + m] = mul_tw(sadd(sadd(a, bk1), ck2), tw[n]);
    x[base + 2 * m] = mul_tw(sadd(sadd(a, bk2), ck1), tw[m + n]);
  } else {
    const c16 a = sra(x[base], 3), b = sra(x[base + m], 3), c = sra(x[base + 2 * m], 3), d = sra(x[base + 3 * m], 3),
              e = sra(x[base + 4 * m], 3);
    auto k1 = [](c16 v) { return mul_shift(v, 10126, -31164); };
    auto k2 = [](c16 v) { return mul_shift(v, -26510, -19261); };
    auto k3 = [](c16 v) { return mul_shift(v, -26510, 19261); };
    auto k4 = [](c16 v) { return mul_shift(v, 10126, 31164); };
    x[base] = sadd(sadd(sadd(a, b), sadd(c, d)), e);
    x[base + m] = mul_tw(sadd(sadd(sadd(a, k1(b)), sadd(k2(c), k3(d))), k4(e)), tw[n]);
    x[base + 2 * m] = mul_tw(sadd(sadd(sadd(a, k2(b)), sadd(k4(c), k1(d))), k3(e)), tw[m + n]);
    x[base + 3 * m] = mul_tw(sadd(sadd(sadd(a, k3(b)), sadd(k1(c), k4(d))), k2(e)), tw[2 * m + n]);
    x[base + 4 * m] = mul_tw(sadd(sadd(sadd(a, k4(b)), sadd(k3(c), k2(d))), k1(e)), tw[3 * m + n]);
  }
}

const zrx::FftPlans& plans() {
  static const zrx::FftPlans P = zrx::fftn_build_plans();
  return P;
}

void fft_plan(const zrx::FftPlan& P, const zrx::FftPlans& R, const c16* in, c16* out) {
  const int N = P.N;
  c16 x[zrx::kFftMaxN];
  std::memcpy(x, in, (size_t)N * sizeof(c16));       // FFTSafe: the input is copied first, so in/out may alias
  for (int s = 0; s < P.nst; s++) {
    const zrx::FftStage st = P.st[s];
    if (st.radix == 0) {
      for (int blk = 0; blk < N / st.M; blk++) (st.M == 4 ? fft4 : fft8)(x + blk * st.M);
    } else {
      const int m = st.M / st.radix;
      const uint32_t* tw = R.tw.data() + st.tw;
      for (int blk = 0; blk < N / st.M; blk++)
        for (int n = 0; n < m; n++) butterfly(x, st.radix, blk * st.M + n, m, n, tw);
    }
  }
  const uint16_t* pos = R.pos.data() + P.pos;
  for (int f = 0; f < N; f++) out[f] = x[pos[f]];
}

// ---- FFT64 on AVX2: 8 complex16 per ymm (re, im interleaved int16) ----------------------
// Stage semantics as above; a radix-4 stage of FFTSSE<N> works on 4 quarter rows, i.e. the
// same butterfly across whole registers (the reference's 4-per-xmm loop, 8 per ymm here).
// mul_j: (re, im) -> (~im, re)
__attribute__((target("avx2"))) inline __m256i mulj_v(__m256i a) {
  const __m256i sw = _mm256_shufflelo_epi16(_mm256_shufflehi_epi16(a, 0xB1), 0xB1);   // (im, re)
  return _mm256_xor_si256(sw, _mm256_set1_epi32(0x0000FFFF));                        // (~im, re)
}
// mul_shift by per-element twiddles w = (re, im) packed like the data: madd_epi16 with
// (bre, ~bim) and (bim, bre), srai 15, pack the low 16 bits of both 32-bit results
__attribute__((target("avx2"))) inline __m256i mul_shift_v(__m256i a, __m256i c1, __m256i c2) {
  const __m256i re = _mm256_srai_epi32(_mm256_madd_epi16(a, c1), 15);
  const __m256i im = _mm256_srai_epi32(_mm256_madd_epi16(a, c2), 15);
  return _mm256_blend_epi16(re, _mm256_slli_epi32(im, 16), 0xAA);
}

struct Fft64Tables {
  alignas(32) int16_t t64[3][2][32];   // [k-1][c1|c2][16 twiddles x 2]
  alignas(32) int16_t t16[3][2][16];   // [k-1][c1|c2][8 lanes: n = 0..3 twice] (two 16-blocks per ymm)
  Fft64Tables() {
    for (int k = 1; k <= 3; k++) {
      for (int n = 0; n < 16; n++) {
        const uint32_t w = zrx::fftn_twiddle(64, k, n);
        const int16_t re = (int16_t)(w & 0xFFFF), im = (int16_t)(w >> 16);
        t64[k - 1][0][2 * n] = re; t64[k - 1][0][2 * n + 1] = (int16_t)~im;
        t64[k - 1][1][2 * n] = im; t64[k - 1][1][2 * n + 1] = re;
      }
      for (int l = 0; l < 8; l++) {
        const int n = l & 3;
        const uint32_t w = zrx::fftn_twiddle(16, k, n);
        const int16_t re = (int16_t)(w & 0xFFFF), im = (int16_t)(w >> 16);
        t16[k - 1][0][2 * l] = re; t16[k - 1][0][2 * l + 1] = (int16_t)~im;
        t16[k - 1][1][2 * l] = im; t16[k - 1][1][2 * l + 1] = re;
      }
    }
  }
};

// twiddle registers of the 64- and 16-point stages (functors, not lambdas: a lambda does not
// inherit the enclosing function's target("avx2"))
struct Tw64 {
  const Fft64Tables* T;
  int h;
  __attribute__((target("avx2"))) __m256i operator()(int k, int j) const {
    return _mm256_load_si256((const __m256i*)&T->t64[k - 1][j][16 * h]);
  }
};
struct Tw16 {
  const Fft64Tables* T;
  __attribute__((target("avx2"))) __m256i operator()(int k, int j) const {
    return _mm256_load_si256((const __m256i*)&T->t16[k - 1][j][0]);
  }
};

// The radix-4 butterfly on registers a, b, c, d (quarter rows), twiddles from tab[k-1][0/1]
template <class Tw>
__attribute__((target("avx2"))) inline void r4_v(__m256i& a, __m256i& b, __m256i& c, __m256i& d, Tw tw) {
  a = _mm256_srai_epi16(a, 2); b = _mm256_srai_epi16(b, 2); c = _mm256_srai_epi16(c, 2); d = _mm256_srai_epi16(d, 2);
  const __m256i ac = _mm256_adds_epi16(a, c), bd = _mm256_adds_epi16(b, d);
  const __m256i a_c = _mm256_subs_epi16(a, c), b_d = _mm256_subs_epi16(b, d);
  const __m256i jb = mulj_v(b_d);
  a = _mm256_adds_epi16(ac, bd);
  b = mul_shift_v(_mm256_subs_epi16(ac, bd), tw(2, 0), tw(2, 1));
  c = mul_shift_v(_mm256_subs_epi16(a_c, jb), tw(1, 0), tw(1, 1));
  d = mul_shift_v(_mm256_adds_epi16(a_c, jb), tw(3, 0), tw(3, 1));
}

// FFTSSEEx<4> on the 4 complex16 of each 128-bit lane (as fft4): y = x >> 2, S = (A, B, A, B)
// with A = y0 + y2, B = y1 + y3, D = (L, T, L, T) with L = y0 + ~y2, T = y1 + ~y3; the outputs
// A + B, ~B + A, L + ~jT, L + jT are (A, A, L, L) + (B, ~B, ~jT, jT), all saturating.
__attribute__((target("avx2"))) inline __m256i fft4_v(__m256i v) {
  const __m256i y = _mm256_srai_epi16(v, 2);
  const __m256i a02 = _mm256_shuffle_epi32(y, 0x44), b13 = _mm256_shuffle_epi32(y, 0xEE);   // (y0,y1,y0,y1), (y2,y3,y2,y3)
  const __m256i S = _mm256_adds_epi16(a02, b13);
  const __m256i D = _mm256_adds_epi16(a02, _mm256_xor_si256(b13, _mm256_set1_epi32(-1)));
  const __m256i J = mulj_v(D);
  const __m256i F = _mm256_unpacklo_epi64(_mm256_shuffle_epi32(S, 0x00), _mm256_shuffle_epi32(D, 0x00));
  const __m256i G = _mm256_xor_si256(_mm256_unpacklo_epi64(_mm256_shuffle_epi32(S, 0x55), _mm256_shuffle_epi32(J, 0x55)),
                                     _mm256_setr_epi32(0, -1, -1, 0, 0, -1, -1, 0));
  return _mm256_adds_epi16(F, G);
}

__attribute__((target("avx2"))) void fft64_avx2(const c16* in, c16* out) {
  static const Fft64Tables T;
  alignas(32) c16 x[64];
  __m256i v[8];
  for (int i = 0; i < 8; i++) v[i] = _mm256_loadu_si256((const __m256i*)(in + 8 * i));
  // stage 64: butterfly n over x[n], x[n+16], x[n+32], x[n+48]: registers (i, i+2, i+4, i+6)
  for (int h = 0; h < 2; h++) {
    r4_v(v[h], v[h + 2], v[h + 4], v[h + 6], Tw64{&T, h});
  }
  // stage 16 on each 16-block q (registers 2q, 2q+1): n over x[16q + n + 4r], r = 0..3; with
  // 8 complex per register, quarters r = 0,1 sit in register 2q (halves), r = 2,3 in 2q+1.
  // Gather quarter rows: A = {q0r0, q1r0}, ... two 16-blocks per register.
  for (int p = 0; p < 2; p++) {
    const __m256i u0 = v[4 * p], u1 = v[4 * p + 1], u2 = v[4 * p + 2], u3 = v[4 * p + 3];
    // u0 = blk(2p)[0..7] = r0|r1, u1 = blk(2p)[8..15] = r2|r3, u2/u3 = blk(2p+1)
    __m256i a = _mm256_permute2x128_si256(u0, u2, 0x20);   // r0 of both blocks
    __m256i b = _mm256_permute2x128_si256(u0, u2, 0x31);   // r1
    __m256i c = _mm256_permute2x128_si256(u1, u3, 0x20);   // r2
    __m256i d = _mm256_permute2x128_si256(u1, u3, 0x31);   // r3
    r4_v(a, b, c, d, Tw16{&T});
    v[4 * p] = _mm256_permute2x128_si256(a, b, 0x20);
    v[4 * p + 1] = _mm256_permute2x128_si256(c, d, 0x20);
    v[4 * p + 2] = _mm256_permute2x128_si256(a, b, 0x31);
    v[4 * p + 3] = _mm256_permute2x128_si256(c, d, 0x31);
  }
  // base case FFTSSEEx<4> on the 16 groups of 4: one group per 128-bit lane
  for (int i = 0; i < 8; i++) _mm256_store_si256((__m256i*)(x + 8 * i), fft4_v(v[i]));
  // bFFT64LUTMap: natural-order bin k is x[bitrev6(k)]
  for (int k = 0; k < 64; k++) {
    const int r = ((k & 1) << 5) | ((k & 2) << 3) | ((k & 4) << 1) | ((k & 8) >> 1) | ((k & 16) >> 3) | ((k & 32) >> 5);
    out[k] = x[r];
  }
}

// ------------------------------------------------------------------ Viterbi brick
constexpr uint32_t kTrellisMax = 40000;   // TViterbiCore<TRELLIS_MAX> columns (sora_ext_viterbi.cpp:39)

// Branch-metric selector of new states 2j (x = 0) and 2j + 1 for j = 0..31 from predecessor
// j (branch 0): index (A << 1) | B of the expected code bits (encoding.blk:92-109; A = x ^ p1
// ^ p2 ^ p4 ^ p5, B = x ^ p0 ^ p1 ^ p2 ^ p5).  Branch 1 (p | 32) and x = 1 flip both bits.
struct VitConsts {
  alignas(32) uint8_t idx0[32], idx1[32];
  VitConsts() {
    for (int j = 0; j < 32; j++) {
      const int A = ((j >> 1) ^ (j >> 2) ^ (j >> 4)) & 1, B = (j ^ (j >> 1) ^ (j >> 2)) & 1;
      idx0[j] = (uint8_t)(A << 1 | B);
      idx1[j] = (uint8_t)(idx0[j] ^ 3);
    }
  }
};
const VitConsts kVit;

// bm(v, e) = e ? 14 - 2v : 2v (VIT_MA / VIT_MB, csrc/viterbilut.h:111-285), u8 arithmetic
inline uint32_t bm(uint32_t v, uint32_t e) { return (e ? 14u - 2u * v : 2u * v) & 0xFFu; }
// Branch-metric table T[c], c = (A << 1) | B, of one column, replicated to every dword:
// USE 3 = (a on A, b on B); 1 = a on A only; 2 = a on B only (BranchACS 2-/1-input forms,
// csrc/viterbicore.hpp:343-390; the depuncture of sora_ext_viterbi.cpp:93-110)
template <int USE>
__attribute__((target("avx2"))) inline __m256i bm_table(uint32_t a, uint32_t b) {
  uint32_t t = 0;
  for (uint32_t c = 0; c < 4; c++) {
    const uint32_t A = c >> 1, B = c & 1;
    const uint32_t v = USE == 3 ? bm(a, A) + bm(b, B) : USE == 1 ? bm(a, A) : bm(a, B);
    t |= (v & 0xFFu) << (8 * c);
  }
  return _mm256_set1_epi32((int)t);
}

// One trellis column (branchACSAdvance, csrc/viterbicore.hpp:105-147): new state 2j + x from
// j (branch 0: sum & 0xFE) and j + 32 (branch 1: sum | 1), min_epu8; L = states 0..31, H =
// 32..63.  Returns the column's survivor markers (bit s = metric LSB of state s).
__attribute__((target("avx2"))) inline uint64_t acs(__m256i& L, __m256i& H, __m256i T) {
  const __m256i i0 = _mm256_load_si256((const __m256i*)kVit.idx0), i1 = _mm256_load_si256((const __m256i*)kVit.idx1);
  const __m256i b0 = _mm256_shuffle_epi8(T, i0), b1 = _mm256_shuffle_epi8(T, i1);
  const __m256i fe = _mm256_set1_epi8((char)0xFE), one = _mm256_set1_epi8(1);
  const __m256i n0 = _mm256_min_epu8(_mm256_and_si256(_mm256_add_epi8(L, b0), fe),
                                     _mm256_or_si256(_mm256_add_epi8(H, b1), one));
  const __m256i n1 = _mm256_min_epu8(_mm256_and_si256(_mm256_add_epi8(L, b1), fe),
                                     _mm256_or_si256(_mm256_add_epi8(H, b0), one));
  const __m256i lo = _mm256_unpacklo_epi8(n0, n1), hi = _mm256_unpackhi_epi8(n0, n1);
  L = _mm256_permute2x128_si256(lo, hi, 0x20);
  H = _mm256_permute2x128_si256(lo, hi, 0x31);
  return (uint64_t)(uint32_t)_mm256_movemask_epi8(_mm256_slli_epi16(L, 7)) |
         ((uint64_t)(uint32_t)_mm256_movemask_epi8(_mm256_slli_epi16(H, 7)) << 32);
}

// normalize (csrc/viterbicore.hpp:149-168): subtract min(all 64) & 0xFE
__attribute__((target("avx2"))) inline void normalize(__m256i& L, __m256i& H) {
  const __m256i v = _mm256_min_epu8(L, H);
  __m128i x = _mm_min_epu8(_mm256_castsi256_si128(v), _mm256_extracti128_si256(v, 1));
  x = _mm_min_epu8(x, _mm_srli_si128(x, 8));
  x = _mm_min_epu8(x, _mm_srli_si128(x, 4));
  x = _mm_min_epu8(x, _mm_srli_si128(x, 2));
  x = _mm_min_epu8(x, _mm_srli_si128(x, 1));
  const __m256i s = _mm256_set1_epi8((char)(_mm_cvtsi128_si32(x) & 0xFE));
  L = _mm256_sub_epi8(L, s);
  H = _mm256_sub_epi8(H, s);
}

// traceback (csrc/viterbicore.hpp:170-239).  The start is the argmin of the SIGNED int16 key
// (m << 8) | 4s (SSE2 hmin16, :79-96): the smallest metric byte read as int8, then the lowest
// state; bit 6 of the walk index carries that state's own marker.  Writes output_bits / 8
// bytes to out, filled from the last.
__attribute__((target("avx2"))) void traceback(__m256i L, __m256i H, const uint64_t* surv, uint32_t col,
                                               uint8_t* out, uint64_t output_bits, uint64_t lookahead) {
  const __m256i v = _mm256_min_epi8(L, H);
  __m128i x = _mm_min_epi8(_mm256_castsi256_si128(v), _mm256_extracti128_si256(v, 1));
  x = _mm_min_epi8(x, _mm_srli_si128(x, 8));
  x = _mm_min_epi8(x, _mm_srli_si128(x, 4));
  x = _mm_min_epi8(x, _mm_srli_si128(x, 2));
  x = _mm_min_epi8(x, _mm_srli_si128(x, 1));
  const __m256i mn = _mm256_set1_epi8((char)_mm_cvtsi128_si32(x));
  const uint64_t eq = (uint64_t)(uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(L, mn)) |
                      ((uint64_t)(uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(H, mn)) << 32);
  const uint32_t s = (uint32_t)__builtin_ctzll(eq);
  uint32_t i = s | (uint32_t)((surv[col] >> s) & 1u) << 6;
  uint32_t t = col;
  for (uint64_t k = 0; k < lookahead; k++) {
    t = t ? t - 1 : 0;                                // (the reference reads before column 0 here: UB)
    i = (i >> 1) & 0x3Fu;
    i |= (uint32_t)((surv[t] >> i) & 1u) << 6;
  }
  for (uint64_t byte = output_bits >> 3; byte-- > 0;) {
    uint32_t oc = 0;
    for (int j = 0; j < 8; j++) {
      oc = (oc << 1) | ((i >> 6) & 1u);
      t = t ? t - 1 : 0;
      i = (i >> 1) & 0x3Fu;
      i |= (uint32_t)((surv[t] >> i) & 1u) << 6;
    }
    out[byte] = (uint8_t)oc;
  }
}

// The global, non-reentrant decoder of csrc/sora_ext_viterbi.cpp:39-46 (one TViterbiCore, the
// brick's schedule state); defaults as the reference's statics (frame_length 1500, CR_12,
// depth 256, column 0 initialised by the constructor).
struct Decoder {
  alignas(32) uint8_t m[64];
  std::vector<uint64_t> surv;
  uint32_t tr = 0;
  uint64_t ob = 0;                 // ob_count (unsigned long)
  uint16_t frame_length = 1500;    // unum16: init truncates frame_len as the reference does
  int16_t code_rate = 0;
  uint64_t depth = 256;            // TRELLIS_DEPTH = (size_t)depth
  void reset() {
    if (surv.empty()) surv.assign(kTrellisMax, 0);
    m[0] = 0;
    for (int s = 1; s < 64; s++) m[s] = 48;        // ALL_INIT0 / ALL_INIT (viterbilut.h)
    surv[0] = 0;
    tr = 0;
    ob = 0;
  }
  Decoder() { reset(); }
};
Decoder& dec() {
  static Decoder d;
  return d;
}

// The group loop of __ext_viterbi_brick_decode_fast (csrc/sora_ext_viterbi.cpp:89-151) for
// code rate CR: G soft values per group, whole groups only (the reference reads past the
// end of a partial one), stopping before the trellis buffer would overflow (the reference
// writes past TRELLIS_MAX columns).
template <int CR>
__attribute__((target("avx2"))) uint32_t decode_groups(Decoder& d, const uint8_t* in, int len, uint8_t* bit) {
  constexpr int G = CR == 0 ? 2 : CR == 1 ? 3 : 4;
  constexpr uint32_t steps = CR == 0 ? 1 : CR == 1 ? 2 : 3;
  __m256i L = _mm256_load_si256((const __m256i*)d.m), H = _mm256_load_si256((const __m256i*)(d.m + 32));
  uint64_t* surv = d.surv.data();
  const uint32_t tr_end = (uint32_t)d.frame_length * 8u + 6u;
  uint32_t total = 0;
  for (int k = 0; k + G <= len; k += G) {
    if (d.tr + steps >= kTrellisMax) break;
    surv[d.tr + 1] = acs(L, H, bm_table<3>(in[k], in[k + 1]));
    if (CR >= 1) surv[d.tr + 2] = acs(L, H, bm_table<1>(in[k + 2], 0));
    if (CR == 2) surv[d.tr + 3] = acs(L, H, bm_table<2>(in[k + 3], 0));
    d.tr += steps;
    const uint32_t tr = d.tr;
    if ((tr & 7u) == 0) normalize(L, H);             // LSB markers are unchanged (even subtrahend)
    uint64_t cnt = 0, look = 0;
    if (tr >= tr_end) {
      cnt = (uint32_t)(tr_end - d.ob - 6u);
      look = tr - tr_end;
    } else if ((uint64_t)tr >= d.ob + d.depth + 24u + 6u) {
      const uint64_t remain = ((uint64_t)tr - (d.ob + d.depth + 24u + 6u)) % 8u;
      cnt = (uint32_t)d.depth;
      look = 24u + remain;
    }
    if (cnt) {
      traceback(L, H, surv, tr, bit + total, cnt, look);
      d.ob += cnt;
      total += (uint32_t)(cnt / 8);
    }
  }
  _mm256_store_si256((__m256i*)d.m, L);
  _mm256_store_si256((__m256i*)(d.m + 32), H);
  return total;
}

}  // namespace

// ------------------------------------------------------------------ internal API
namespace zrx_host {

// csrc/sora_ext_lib.cpp:2672-2812: an unsupported size prints and leaves the output untouched
void sora_fft(struct complex16* out, int nfft, const struct complex16* in) {
  if (zrx::fftn_index(nfft) < 0) {
    std::printf("__ext_sora_fft error: fft size %d not supported!\n", nfft);
    return;
  }
  require_avx2();
  if (nfft == 64) {
    fft64_avx2((const c16*)in, (c16*)out);
    return;
  }
  const zrx::FftPlans& R = plans();
  fft_plan(R.plans[zrx::fftn_index(nfft)], R, (const c16*)in, (c16*)out);
}

int vit_init(int32_t frame_len, int16_t code_rate, int16_t depth) {
  Decoder& d = dec();
  d.reset();
  d.frame_length = (uint16_t)frame_len;
  d.code_rate = code_rate;
  d.depth = (uint64_t)(int64_t)depth;
  return 0;
}

int16_t vit_decode(const char* soft, int len, unsigned char* bit) {
  require_avx2();
  Decoder& d = dec();
  const uint8_t* in = (const uint8_t*)soft;         // the brick reads its input as unsigned char
  uint32_t bytes = 0;
  switch (d.code_rate) {
    case 0: bytes = decode_groups<0>(d, in, len, bit); break;
    case 1: bytes = decode_groups<1>(d, in, len, bit); break;
    case 2: bytes = decode_groups<2>(d, in, len, bit); break;
    default: break;                                  // the reference loops forever here
  }
  return (int16_t)(bytes * 8u);
}

// Viterbi_sig11 (csrc/viterbicore.hpp:272-315): 24 rate-1/2 columns from the initial state,
// normalize every 8 and once more at the end, 24-bit traceback, lookahead 0; then the brick's
// *(unum32*)bit >>= 6 (sora_ext_viterbi.cpp:191)
__attribute__((target("avx2"))) void sig_decode(const char* soft48, unsigned char* bit) {
  require_avx2();
  alignas(32) uint8_t m0[64];
  m0[0] = 0;
  for (int s = 1; s < 64; s++) m0[s] = 48;
  __m256i L = _mm256_load_si256((const __m256i*)m0), H = _mm256_load_si256((const __m256i*)(m0 + 32));
  uint64_t surv[25];
  surv[0] = 0;
  const uint8_t* in = (const uint8_t*)soft48;
  for (int t = 1; t <= 24; t++) {
    surv[t] = acs(L, H, bm_table<3>(in[2 * t - 2], in[2 * t - 1]));
    if ((t & 7) == 0) normalize(L, H);
  }
  normalize(L, H);
  traceback(L, H, surv, 24, bit, 24, 0);
  uint32_t w;
  std::memcpy(&w, bit, 4);
  w >>= 6;
  std::memcpy(bit, &w, 4);
}

// __ext_v_shift_right_complex16 (csrc/sora_ext_lib.cpp:1979-1995): the first len/4*4 complex
// values by srai_epi16 (a count above 15 fills with the sign), the tail by unum16 >> shift
int shift_right(struct complex16* z, const struct complex16* x, int len, int shift) {
  if (len <= 0) return 0;
  const int16_t* xs = (const int16_t*)x;
  int16_t* zs = (int16_t*)z;
  const int head = (len / 4) * 8;
  for (int e = 0; e < 2 * len; e++) {
    if (e < head) {
      zs[e] = (shift < 0 || shift > 15) ? (int16_t)(xs[e] < 0 ? -1 : 0) : (int16_t)(xs[e] >> shift);
    } else {
      const uint16_t u = (uint16_t)xs[e];
      zs[e] = (int16_t)((shift < 0 || shift > 15) ? 0 : (u >> shift));
    }
  }
  return 0;
}

}  // namespace zrx_host

// ------------------------------------------------------------------ C linkage (ctypes, C callers)
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
  (void)len2;                                        // the reference does not bound its writes either
  return zrx_host::vit_decode(intInput, len1, bit);
}
int __ext_viterbiSig11a_brick_init_fast(int32_t frame_len, int16_t code_rate, int16_t depth) {
  return zrx_host::vit_init(frame_len, code_rate, depth);   // resets the same global decoder (:159-173)
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
