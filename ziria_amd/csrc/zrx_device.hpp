// Device building blocks of the MI355X 802.11a RX engine (gfx950, wave64).
//
// Bit-exactness contract: every routine reproduces the reference bricks' integer
// semantics exactly (SSE2 saturating int16 adds, XOR-as-negate, madd_epi16 32-bit wrap,
// u8 wrapping Viterbi metrics with the survivor marker in the metric LSB, signed-int16
// traceback key).  Reference lines are cited per routine (paths relative to moxfun/Ziria).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "zrx_tables.h"

namespace zrx {

typedef short s2 __attribute__((ext_vector_type(2)));   // one complex16 = (re, im)

__device__ __forceinline__ s2 as_s2(uint32_t v) { return __builtin_bit_cast(s2, v); }
__device__ __forceinline__ uint32_t as_u32(s2 v) { return __builtin_bit_cast(uint32_t, v); }

// ------------------------------------------------------------------ FFT64 (lane = symbol)
// _mm_adds_epi16 / _mm_subs_epi16 -> v_pk_add_i16 / v_pk_sub_i16 with clamp.
__device__ __forceinline__ s2 sat_add(s2 a, s2 b) { return __builtin_elementwise_add_sat(a, b); }
__device__ __forceinline__ s2 sat_sub(s2 a, s2 b) { return __builtin_elementwise_sub_sat(a, b); }
__device__ __forceinline__ s2 shr2(s2 a) { return a >> (s2){2, 2}; }               // srai 2
// mul_jx (csrc/sora_ext_lib_fft.hpp:98-108): (re, im) -> (~im, re)
__device__ __forceinline__ s2 mul_j(s2 a) { return (s2){(short)~a.y, a.x}; }
// mul_shiftx(a, b, 15) (csrc/sora_ext_lib_fft.hpp:42-67): madd_epi16 = v_dot2 (32-bit
// wrapping sum of two exact products), srai 15, low 16 bits.
__device__ __forceinline__ s2 mul_shift(s2 a, short bre, short bim) {
  const s2 c1 = {bre, (short)~bim}, c2 = {bim, bre};
  const int re = __builtin_amdgcn_sdot2(a, c1, 0, false);
  const int im = __builtin_amdgcn_sdot2(a, c2, 0, false);
  return (s2){(short)(re >> 15), (short)(im >> 15)};
}

// FFTSSE<N> (csrc/fft_r4difx.hpp:54-97): one radix-4 DIF stage in place.
template <int N>
__device__ __forceinline__ void fft_stage(s2* x) {
  const int16_t* t1 = N == 64 ? kTw64_1 : kTw16_1;
  const int16_t* t2 = N == 64 ? kTw64_2 : kTw16_2;
  const int16_t* t3 = N == 64 ? kTw64_3 : kTw16_3;
#pragma unroll
  for (int n = 0; n < N / 4; n++) {
    const s2 a = shr2(x[n]), b = shr2(x[n + N / 4]), c = shr2(x[n + N / 2]), d = shr2(x[n + 3 * N / 4]);
    const s2 ac = sat_add(a, c), bd = sat_add(b, d), a_c = sat_sub(a, c), b_d = sat_sub(b, d);
    x[n] = sat_add(ac, bd);
    x[n + N / 4] = mul_shift(sat_sub(ac, bd), t2[2 * n], t2[2 * n + 1]);
    const s2 jb = mul_j(b_d);
    x[n + N / 2] = mul_shift(sat_sub(a_c, jb), t1[2 * n], t1[2 * n + 1]);
    x[n + 3 * N / 4] = mul_shift(sat_add(a_c, jb), t3[2 * n], t3[2 * n + 1]);
  }
}
// FFTSSEEx<4> (csrc/fft_r4difx.hpp:111-140), regrouped on packed (re, im) pairs:
// A = y0+y2, B = y1+y3, L = y0+~y2, T = y1+~y3 (saturating); outputs A+B, ~B+A,
// L+~j(T), L+j(T) — identical lane-for-lane to the XOR/shuffle sequence.
__device__ __forceinline__ void fft4(s2* x) {
  const s2 y0 = shr2(x[0]), y1 = shr2(x[1]), y2 = shr2(x[2]), y3 = shr2(x[3]);
  const s2 A = sat_add(y0, y2), B = sat_add(y1, y3);
  const s2 L = sat_add(y0, ~y2), T = sat_add(y1, ~y3);
  const s2 jT = mul_j(T);
  x[0] = sat_add(A, B);
  x[1] = sat_add(~B, A);
  x[2] = sat_add(L, ~jT);
  x[3] = sat_add(L, jT);
}
__host__ __device__ constexpr int bitrev6(int i) {
  return ((i & 1) << 5) | ((i & 2) << 3) | ((i & 4) << 1) | ((i & 8) >> 1) | ((i & 16) >> 3) | ((i & 32) >> 5);
}
// FFTSSEEx<64> in place; natural-order output bin k lives at x[bitrev6(k)]
// (bFFT64LUTMap, csrc/sora_ext_lib_fft_coeffs.hpp:15090-15094).
__device__ __forceinline__ void fft64_inplace(s2* x) {
  fft_stage<64>(x);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    fft_stage<16>(x + 16 * q);
#pragma unroll
    for (int r = 0; r < 4; r++) fft4(x + 16 * q + 4 * r);
  }
}

// ------------------------------------------------------------------ GetData + demap + deinterleave
// GetData.blk:24-35: data bins 38..42, 44..56, 58..63, 1..6, 8..20, 22..26
__host__ __device__ constexpr int data_bin(int i) {
  return i < 5 ? 38 + i : i < 18 ? 44 + (i - 5) : i < 24 ? 58 + (i - 18) : i < 30 ? 1 + (i - 24)
       : i < 43 ? 8 + (i - 30) : 22 + (i - 43);
}
template <int MOD> struct ModInfo;
template <> struct ModInfo<0> { static constexpr int nb = 1, ncbps = 48; };
template <> struct ModInfo<1> { static constexpr int nb = 2, ncbps = 96; };
template <> struct ModInfo<2> { static constexpr int nb = 4, ncbps = 192; };
template <> struct ModInfo<3> { static constexpr int nb = 6, ncbps = 288; };
template <int MOD>
__host__ __device__ constexpr int deint_src(int k) {
  return MOD == 0 ? kDeint48[k] : MOD == 1 ? kDeint96[k] : MOD == 2 ? kDeint192[k] : kDeint288[k];
}
// Demap*.blk:22-33 soft order per subcarrier -> (component 0 = re / 1 = im, LUT byte).
// LUT bytes: 0 m_bpsk_lut, 1 m_qam16_lut2, 2 m_qam64_lut2, 3 m_qam64_lut3.
template <int MOD>
__host__ __device__ constexpr int soft_comp(int c) {
  return MOD == 0 ? 0 : MOD == 1 ? c : MOD == 2 ? (c >> 1) : (c >= 3 ? 1 : 0);
}
template <int MOD>
__host__ __device__ constexpr int soft_lutbyte(int c) {
  return MOD <= 1 ? 0 : MOD == 2 ? (c & 1) : (c % 3 == 0 ? 0 : (c % 3 == 1 ? 2 : 3));
}

// DemapLimit (DemapLimit.blk:22-63, shift 0): clip to [-128,127]; the u8 LUT index is the
// low byte of the clipped value.  lut: kDemapLut staged in LDS.
// Writes ncbps soft bytes (deinterleaved, Deinterleave*.blk) as ncbps/4 words.
template <int MOD>
__device__ __forceinline__ void demap_deinterleave(const s2* x, const uint32_t* lut, uint32_t* w) {
  constexpr int NB = ModInfo<MOD>::nb, NC = ModInfo<MOD>::ncbps;
  uint32_t lr[48], li[48];
#pragma unroll
  for (int i = 0; i < 48; i++) {
    s2 v = x[bitrev6(data_bin(i))];
    v = __builtin_elementwise_max(__builtin_elementwise_min(v, (s2){127, 127}), (s2){-128, -128});
    const uint32_t u = as_u32(v);
    lr[i] = lut[u & 0xFF];
    li[i] = (MOD == 0) ? 0u : lut[(u >> 16) & 0xFF];
  }
#pragma unroll
  for (int d = 0; d < NC / 4; d++) {
    uint32_t word = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const int j = deint_src<MOD>(4 * d + b);
      const int i = j / NB, c = j % NB;
      const uint32_t src = soft_comp<MOD>(c) ? li[i] : lr[i];
      word |= ((src >> (8 * soft_lutbyte<MOD>(c))) & 0xFFu) << (8 * b);
    }
    w[d] = word;
  }
}

// demap_deinterleave that hands each group of 4 words (16 soft bytes) to st(q, uint4) as
// soon as it is built, so the whole soft symbol never has to be live in registers.
// lut(i) returns kDemapLut[i] (k_data_fft reads one of several LDS copies per lane).
// Each output dword takes its 4 soft bytes from 4 different subcarrier components (the
// deinterleaver spreads neighbours), and each LUT dword holds the soft values as whole bytes,
// so a word is two byte gathers (v_perm, the other bytes zero) and an OR.
template <int MOD, int K>
__host__ __device__ constexpr uint32_t soft_src(int b) {   // (register id i*2+comp) of byte b of word K
  return (uint32_t)(2 * (deint_src<MOD>(4 * K + b) / ModInfo<MOD>::nb) + soft_comp<MOD>(deint_src<MOD>(4 * K + b) % ModInfo<MOD>::nb));
}
template <int MOD, int K>
__host__ __device__ constexpr uint32_t soft_byte(int b) {  // LUT byte of byte b of word K
  return (uint32_t)soft_lutbyte<MOD>(deint_src<MOD>(4 * K + b) % ModInfo<MOD>::nb);
}
// v_perm selector placing byte lo of S1 at position b0 and byte hi of S0 at position b1, zeros elsewhere
__host__ __device__ constexpr uint32_t perm_sel2(int b0, uint32_t lo, int b1, uint32_t hi) {
  uint32_t s = 0x0C0C0C0Cu;
  s &= ~(0xFFu << (8 * b0)); s |= lo << (8 * b0);
  s &= ~(0xFFu << (8 * b1)); s |= (4u + hi) << (8 * b1);
  return s;
}
template <int MOD, int K>
__device__ __forceinline__ uint32_t soft_word(const uint32_t* lr, const uint32_t* li) {
  auto reg = [&](uint32_t id) { return (id & 1u) ? li[id >> 1] : lr[id >> 1]; };
  const uint32_t a = __builtin_amdgcn_perm(reg(soft_src<MOD, K>(1)), reg(soft_src<MOD, K>(0)),
                                           perm_sel2(0, soft_byte<MOD, K>(0), 1, soft_byte<MOD, K>(1)));
  const uint32_t b = __builtin_amdgcn_perm(reg(soft_src<MOD, K>(3)), reg(soft_src<MOD, K>(2)),
                                           perm_sel2(2, soft_byte<MOD, K>(2), 3, soft_byte<MOD, K>(3)));
  return a | b;
}
template <int MOD, int Q, class St>
__device__ __forceinline__ void soft_unit(const uint32_t* lr, const uint32_t* li, St& st) {
  st(Q, make_uint4(soft_word<MOD, 4 * Q>(lr, li), soft_word<MOD, 4 * Q + 1>(lr, li), soft_word<MOD, 4 * Q + 2>(lr, li),
                   soft_word<MOD, 4 * Q + 3>(lr, li)));
}
template <int MOD, class St, int... Q>
__device__ __forceinline__ void soft_units(const uint32_t* lr, const uint32_t* li, St& st, std::integer_sequence<int, Q...>) {
  (soft_unit<MOD, Q>(lr, li, st), ...);
}
template <int MOD, class Lut, class St>
__device__ __forceinline__ void demap_deinterleave_st(const s2* x, Lut lut, St st) {
  constexpr int NC = ModInfo<MOD>::ncbps;
  uint32_t lr[48], li[48];
#pragma unroll
  for (int i = 0; i < 48; i++) {
    s2 v = x[bitrev6(data_bin(i))];
    v = __builtin_elementwise_max(__builtin_elementwise_min(v, (s2){127, 127}), (s2){-128, -128});
    const uint32_t u = as_u32(v);
    lr[i] = lut(u & 0xFF);
    li[i] = (MOD == 0) ? 0u : lut((u >> 16) & 0xFF);
  }
  soft_units<MOD>(lr, li, st, std::make_integer_sequence<int, NC / 16>{});
}
// The same in two steps, so that a wave whose lanes mix modulations reads the LUT once: the
// LUT words of both components of the 48 data bins (a BPSK lane's li go unused: the LUT
// index is the clipped component whatever the modulation), then the packing of MOD.
template <class Lut>
__device__ __forceinline__ void demap_lut_words(const s2* x, Lut lut, uint32_t (&lr)[48], uint32_t (&li)[48]) {
#pragma unroll
  for (int i = 0; i < 48; i++) {
    s2 v = x[bitrev6(data_bin(i))];
    v = __builtin_elementwise_max(__builtin_elementwise_min(v, (s2){127, 127}), (s2){-128, -128});
    const uint32_t u = as_u32(v);
    lr[i] = lut(u & 0xFF);
    li[i] = lut((u >> 16) & 0xFF);
  }
}
template <int MOD, class St>
__device__ __forceinline__ void demap_pack_st(const uint32_t (&lr)[48], const uint32_t (&li)[48], St st) {
  soft_units<MOD>(lr, li, st, std::make_integer_sequence<int, ModInfo<MOD>::ncbps / 16>{});
}

// ------------------------------------------------------------------ ChannelEqualization + PilotTrack
// (receiver.blk:68-69).  Trig tables live in HBM, built once by the host
// (zrx_api.hip) from the closed forms of the reference LUTs (csrc/intalglutx.h):
// rot[r] = (cosx(r), -sinx(r)) as one complex16, atan[(u8)y << 8 | (u8)x] = atan2x_lut.
struct EqTabs {
  const uint32_t* __restrict__ rot;
  const int16_t* __restrict__ atan;
};
// __ext_v_mul_complex16 (csrc/sora_ext_lib.cpp:2098-2137) on one complex16: im negated in
// 16 bits, madd_epi16 = v_dot2 (two exact products, 32-bit wrapping sum), >> sh, low 16 bits.
__device__ __forceinline__ s2 vmul_c16(s2 x, s2 y, int sh) {
  const s2 a = {x.x, (short)-x.y}, b = {x.y, x.x};
  const int re = __builtin_amdgcn_sdot2(a, y, 0, false);
  const int im = __builtin_amdgcn_sdot2(b, y, 0, false);
  return (s2){(short)(re >> sh), (short)(im >> sh)};
}
// atan2x (csrc/intalgx.h:88-99): common right shift until |y|, |x| < 128, then the table.
__device__ __forceinline__ int atan2_16(int y, int x, const int16_t* __restrict__ tab) {
  const uint32_t ay = (uint32_t)abs(y), ax = (uint32_t)abs(x);
  const int ys = ay ? 31 - __builtin_clz(ay) : 0, xs = ax ? 31 - __builtin_clz(ax) : 0;
  const int sh = max(xs, ys) - 6;
  if (sh > 0) { y >>= sh; x >>= sh; }
  return tab[((uint32_t)(y & 0xFF) << 8) | (uint32_t)(x & 0xFF)];
}
__device__ __forceinline__ s2 neg16(s2 v) { return (s2){(short)-v.x, (short)-v.y}; }
// PilotTrack.blk:117-203 on symbol k of a packet (k = 0: SIGNAL; symbol_count starts at 127)
// from its four equalized pilots (bins 43, 57, 7, 21): the common phase `avg` and the slope
// `del`; build_coeff (:28-50) then rotates bin b by angle avg + s(b) * del (mod 2^16), with
// s(b) = b for b in 1..26 and b - 64 for b in 38..63.
__device__ __forceinline__ void pilot_phase(s2 p1, s2 p2, s2 p3, s2 p4, int k, const int16_t* __restrict__ tab,
                                            int& avg, int& del) {
  const int sc = k == 0 ? 127 : (k - 1) % 127;
  if ((kPilotNeg[sc >> 5] >> (sc & 31)) & 1u) { p1 = neg16(p1); p2 = neg16(p2); p3 = neg16(p3); p4 = neg16(p4); }
  int th0 = atan2_16(p1.y, p1.x, tab), th1 = atan2_16(p2.y, p2.x, tab);
  int th2 = atan2_16(p3.y, p3.x, tab), th3 = atan2_16((short)-p4.y, (short)-p4.x, tab);
  // phase unwrap along the pilots (:186-196)
  if (th0 - th1 > 32768) th1 += 65536; else if (th1 - th0 > 32768) th1 -= 65536;
  if (th1 - th2 > 32768) th2 += 65536; else if (th2 - th1 > 32768) th2 -= 65536;
  if (th2 - th3 > 32768) th3 += 65536; else if (th3 - th2 > 32768) th3 -= 65536;
  const int a32 = (th0 + th1 + th2 + th3) / 4;
  avg = a32 >= 32768 ? a32 - 65536 : a32 <= -32768 ? a32 + 65536 : (int)(short)a32;
  del = (short)(((th2 - th0) / 28 + (th3 - th1) / 28) >> 1);
}
__device__ __forceinline__ s2 rot_coeff(int avg, int del, int b, const uint32_t* __restrict__ rot) {
  const int sb = b < 32 ? b : b - 64;
  return as_s2(rot[(uint32_t)(avg + sb * del) & 0xFFFFu]);
}
// FFT output x (bin b at x[bitrev6(b)]) -> ChannelEqualization -> PilotTrack on the bins
// GetData keeps (the other bins are never read downstream).  C(b): channel coefficient.
template <class Coef>
__device__ __forceinline__ void equalize_data_bins(s2* x, const Coef& C, int k, const EqTabs& T) {
  const s2 p1 = vmul_c16(x[bitrev6(43)], C(43), 8), p2 = vmul_c16(x[bitrev6(57)], C(57), 8);
  const s2 p3 = vmul_c16(x[bitrev6(7)], C(7), 8), p4 = vmul_c16(x[bitrev6(21)], C(21), 8);
  int avg, del;
  pilot_phase(p1, p2, p3, p4, k, T.atan, avg, del);
#pragma unroll
  for (int i = 0; i < 48; i++) {
    const int b = data_bin(i);
    const s2 e = vmul_c16(x[bitrev6(b)], C(b), 8);
    x[bitrev6(b)] = vmul_c16(e, rot_coeff(avg, del, b, T.rot), 15);
  }
}

// ------------------------------------------------------------------ wave reductions
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}
__device__ __forceinline__ int wave_min_i32(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ uint32_t wave_xor_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v ^= (uint32_t)__shfl_xor((int)v, o);
  return v;
}
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o);
  return v;
}

// ------------------------------------------------------------------ descrambler / CRC helpers
// CRC register after processing n zero bytes (linear map), via kCrcZero[k] = 2^k bytes.
__device__ __forceinline__ uint32_t crc_apply(const uint32_t* M, uint32_t v) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) r ^= ((v >> i) & 1u) ? M[i] : 0u;
  return r;
}

}  // namespace zrx
