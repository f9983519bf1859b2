// TX chain: transmitter() of code/WiFi/transmitter/transmitter.blk:128-133
// at its default 40 MHz oversampling (FFT_SIZE 128, CP_SIZE 32, ifft.blk), batched over packets.
//
//   k_tx  one wave per packet, lane = OFDM symbol (0 = SIGNAL): the packet's bit stream
//         (SERVICE, payload, CRC-32, pad; crc.blk / tx_driver :56-101) scrambled with the
//         127-periodic keystream of state 1011101 (scramble.blk), convolutionally encoded and
//         punctured (encoding.blk) for the lane's symbol, interleaved (interleaving.blk) through
//         LDS, mapped (modulating.blk), placed with the pilots (map_ofdm.blk) in the 128-bin
//         spectrum, IFFT<128> (csrc/ifft_r4difx.hpp) and cyclic prefix (ifft.blk:35-52); the
//         640-sample preamble (createPreamble.blk) is a host-built constant copied per packet.
#pragma once
#include "zrx_device.hpp"

namespace zrx {
namespace tx {

// conj_mul_shiftx(a, b, 15) (csrc/sora_ext_lib_fft.hpp:68-94): a * conj(b), a.re complemented
// in the imaginary part, madd_epi16 with 32-bit wrap, >> 15, low 16 bits
__device__ __forceinline__ s2 conj_mul_shift(s2 a, short br, short bi) {
  const int re = __builtin_amdgcn_sdot2(a, (s2){br, bi}, 0, false);
  const int im = __builtin_amdgcn_sdot2((s2){a.y, (short)~a.x}, (s2){br, bi}, 0, false);
  return (s2){(short)(re >> 15), (short)(im >> 15)};
}
// IFFTSSE<N> (ifft_r4difx.hpp:56-97)
template <int N>
__device__ __forceinline__ void ifft_stage(s2* x) {
  const int16_t* t1 = N == 128 ? kTw128_1 : kTw32_1;
  const int16_t* t2 = N == 128 ? kTw128_2 : kTw32_2;
  const int16_t* t3 = N == 128 ? kTw128_3 : kTw32_3;
#pragma unroll
  for (int n = 0; n < N / 4; n++) {
    const s2 a = shr2(x[n]), b = shr2(x[n + N / 4]), c = shr2(x[n + N / 2]), d = shr2(x[n + 3 * N / 4]);
    const s2 ac = sat_add(a, c), bd = sat_add(b, d), a_c = sat_sub(a, c), b_d = sat_sub(b, d);
    x[n] = sat_add(ac, bd);
    x[n + N / 4] = conj_mul_shift(sat_sub(ac, bd), t2[2 * n], t2[2 * n + 1]);
    const s2 jb = mul_j(b_d);
    x[n + N / 2] = conj_mul_shift(sat_add(a_c, jb), t1[2 * n], t1[2 * n + 1]);
    x[n + 3 * N / 4] = conj_mul_shift(sat_sub(a_c, jb), t3[2 * n], t3[2 * n + 1]);
  }
}
// IFFTSSEEx<8> (ifft_r4difx.hpp:152-228)
__device__ __forceinline__ void ifft8(s2* x) {
  s2 s[4], e[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const s2 a = x[k] >> (s2){3, 3}, b = x[k + 4] >> (s2){3, 3};
    s[k] = sat_add(a, b);
    e[k] = sat_sub(a, b);
  }
  const s2 A = sat_add(s[0], s[2]), B = sat_add(s[1], s[3]);
  const s2 C = sat_add(~s[2], s[0]), D = sat_add(~s[3], s[1]);
  const s2 jD = mul_j(D);
  x[0] = sat_add(A, B);
  x[1] = sat_add(~B, A);
  x[2] = sat_add(C, jD);
  x[3] = sat_add(~jD, C);
  const s2 je2 = mul_j(e[2]), je3 = mul_j(e[3]);
  const s2 u0 = conj_mul_shift(sat_add(e[0], je2), 32767, 0);
  const s2 u1 = conj_mul_shift(sat_add(e[1], je3), 23169, -23169);
  const s2 u2 = conj_mul_shift(sat_add(~je2, e[0]), 32767, 0);
  const s2 u3 = conj_mul_shift(sat_add(~je3, e[1]), -23169, -23169);
  x[4] = sat_add(u0, u1);
  x[5] = sat_add(~u1, u0);
  x[6] = sat_add(u2, u3);
  x[7] = sat_add(~u3, u2);
}
__host__ __device__ constexpr int bitrev7(int i) {
  return ((i & 1) << 6) | ((i & 2) << 4) | ((i & 4) << 2) | (i & 8) | ((i & 16) >> 2) | ((i & 32) >> 4) | ((i & 64) >> 6);
}
// IFFT<128> in place; natural-order output sample t at x[bitrev7(t)] (FFT128LUTMap)
__device__ __forceinline__ void ifft128_inplace(s2* x) {
  ifft_stage<128>(x);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    ifft_stage<32>(x + 32 * q);
#pragma unroll
    for (int r = 0; r < 4; r++) ifft8(x + 32 * q + 8 * r);
  }
}

// modulating.blk (bpsk_mod_11a = 10720 and derived, const.blk:29-32), bits in stream order
template <int MOD>
__device__ __forceinline__ s2 map_bits(const uint8_t* b) {
  if constexpr (MOD == 0) return (s2){(short)(b[0] ? 10720 : -10720), 0};
  if constexpr (MOD == 1) return (s2){(short)(b[0] ? 7581 : -7581), (short)(b[1] ? 7581 : -7581)};
  if constexpr (MOD == 2) {
    const int g0 = b[0] ? (b[1] ? 1 : 3) : (b[1] ? -1 : -3), g1 = b[2] ? (b[3] ? 1 : 3) : (b[3] ? -1 : -3);
    return (s2){(short)(g0 * 3390), (short)(g1 * 3390)};
  }
  const int i0 = b[0] * 4 + b[1] * 2 + b[2], i1 = b[3] * 4 + b[4] * 2 + b[5];
  const int g0 = (i0 & 4 ? 1 : -1) * ((i0 & 3) == 0 ? 7 : (i0 & 3) == 1 ? 5 : (i0 & 3) == 2 ? 1 : 3);
  const int g1 = (i1 & 4 ? 1 : -1) * ((i1 & 3) == 0 ? 7 : (i1 & 3) == 1 ? 5 : (i1 & 3) == 2 ? 1 : 3);
  return (s2){(short)(g0 * 1654), (short)(g1 * 1654)};
}
template <int MOD>
__device__ __forceinline__ int intlv(int j) {
  return MOD == 0 ? kIntlv48[j] : MOD == 1 ? kIntlv96[j] : MOD == 2 ? kIntlv192[j] : kIntlv288[j];
}

// Packet bit b of the scrambled stream: SERVICE (16 zeros), payload (LSB first), CRC-32, pad,
// XOR the keystream of state 1011101 (127-periodic, kTxKey bit (b mod 127)).
struct Stream {
  const uint8_t* __restrict__ pay;
  int plen;
  uint32_t crc;
  __device__ __forceinline__ uint32_t raw(int b) const {
    const int p = b - 16;
    if (p < 0) return 0u;
    if (p < 8 * plen) return (pay[p >> 3] >> (p & 7)) & 1u;
    const int c = p - 8 * plen;
    return c < 32 ? (crc >> c) & 1u : 0u;
  }
  __device__ __forceinline__ uint32_t bit(int b) const {
    const int m = b % 127, w = m >> 5;                 // keystream word by selects, not a load
    const uint32_t key = w == 0 ? kTxKey[0] : w == 1 ? kTxKey[1] : w == 2 ? kTxKey[2] : kTxKey[3];
    return raw(b) ^ ((key >> (m & 31)) & 1u);
  }
};

// coded bits of one symbol into LDS (stream order), then interleave + map into 48 subcarriers
template <int MOD>
__device__ __forceinline__ void symbol_bits(const Stream& S, int first_bit, int nd, int coding, uint8_t* cb, s2* sub) {
  constexpr int NC = ModInfo<MOD>::ncbps, NB = ModInfo<MOD>::nb;
  uint32_t sr = 0;                                        // previous 6 bits, bit j = s[j] (encoding.blk)
  for (int j = 6; j >= 1; j--) sr = (sr << 1) | (first_bit - j >= 0 ? S.bit(first_bit - j) : 0u);
  int k = 0;
  for (int i = 0; i < nd; i++) {
    const uint32_t b = S.bit(first_bit + i);
    const uint32_t A = (b ^ (sr >> 1) ^ (sr >> 2) ^ (sr >> 4) ^ (sr >> 5)) & 1u;
    const uint32_t B = (b ^ sr ^ (sr >> 1) ^ (sr >> 2) ^ (sr >> 5)) & 1u;
    sr = ((sr << 1) | b) & 63u;
    if (coding == 0) { cb[k++] = (uint8_t)A; cb[k++] = (uint8_t)B; }
    else if (coding == 2) {                               // encode34: A0 B0 | A1 | B2
      const int ph = i % 3;
      if (ph == 0) { cb[k++] = (uint8_t)A; cb[k++] = (uint8_t)B; }
      else if (ph == 1) cb[k++] = (uint8_t)A;
      else cb[k++] = (uint8_t)B;
    } else {                                              // encode23: A0 B0 | A1
      if ((i & 1) == 0) { cb[k++] = (uint8_t)A; cb[k++] = (uint8_t)B; }
      else cb[k++] = (uint8_t)A;
    }
  }
#pragma unroll
  for (int i = 0; i < 48; i++) {
    uint8_t b[6];
#pragma unroll
    for (int c = 0; c < NB; c++) b[c] = cb[intlv<MOD>(NB * i + c)];
    sub[i] = map_bits<MOD>(b);
  }
  (void)NC;
}

// CRC-32 of the payload (crc.blk: reflected, init all ones, final inversion), one lane
__device__ __forceinline__ uint32_t crc32_bytes(const uint8_t* __restrict__ p, int n) {
  uint32_t c = 0xFFFFFFFFu;
  for (int i = 0; i < n; i++) c = (c >> 8) ^ kCrcTab[(c ^ p[i]) & 0xFFu];
  return ~c;
}

// The same CRC by the whole wave (n <= 2048): lane l takes the 32-byte chunk l of the n
// bytes right-aligned in a 2048-byte frame (chunks before the data are zero and leave a
// zero-initialised register at zero; the all-ones init is folded in by complementing the
// first 4 data bytes), runs slicing-by-4 (kCrcS4) over it, advances the result past the
// 63 - l chunks behind it with the 32·2^k-zero-byte maps (kCrcShift), and the wave XORs the
// partial registers -- the k_descramble_crc scheme without the descrambler.
__device__ __forceinline__ uint32_t crc32_wave(const uint8_t* __restrict__ p, int n, int lane) {
  if (n < 4) return (uint32_t)__builtin_amdgcn_readfirstlane((int)crc32_bytes(p, n));
  const int q0 = 32 * lane - (2048 - n);                // data index of this lane's first byte
  uint32_t r = 0;
  if (q0 + 32 > 0) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint32_t x = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const int q = q0 + 4 * j + b;
        uint32_t v = q >= 0 ? (uint32_t)p[max(q, 0)] : 0u;
        if (q >= 0 && q < 4) v ^= 0xFFu;
        x |= v << (8 * b);
      }
      r ^= x;
      r = kCrcS4[3][r & 0xFFu] ^ kCrcS4[2][(r >> 8) & 0xFFu] ^ kCrcS4[1][(r >> 16) & 0xFFu] ^ kCrcS4[0][r >> 24];
    }
    const uint32_t adv = 63u - (uint32_t)lane;
#pragma unroll
    for (int k = 0; k < 6; k++) {
      uint32_t t = 0;
#pragma unroll
      for (int j = 0; j < 8; j++) t ^= kCrcShift[k][j * 16 + ((r >> (4 * j)) & 15u)];
      if ((adv >> k) & 1u) r = t;
    }
  }
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)~wave_xor_u32(r));
}

// in: per packet 3 PLCP header bytes (emitHeader, parsePLCPHeader.blk:215-221) then len-4
// payload bytes; out: 640 + 160 * (1 + nsym) complex16 samples at out_off[p].
__global__ __launch_bounds__(64) void k_tx(const uint8_t* __restrict__ in, const int64_t* __restrict__ in_off,
                                           int npkts, const uint32_t* __restrict__ preamble,
                                           uint32_t* __restrict__ out, const int64_t* __restrict__ out_off,
                                           int32_t* __restrict__ nsamp) {
  __shared__ uint8_t lds[64 * 288];
  __shared__ uint8_t pay[2048];                           // the payload, read bit by bit below
  const int lane = threadIdx.x;
  const int p = blockIdx.x;
  if (p >= npkts) return;
  const uint8_t* src = in + in_off[p];
  const uint32_t hb = (uint32_t)src[0] | ((uint32_t)src[1] << 8) | ((uint32_t)src[2] << 16);
  int mod = 0, cod = 0;                                   // parsePLCPHeader.blk:124-158
  switch (hb & 0xF) {
    case 0xB: mod = 0; cod = 0; break;
    case 0xF: mod = 0; cod = 2; break;
    case 0xA: mod = 1; cod = 0; break;
    case 0xE: mod = 1; cod = 2; break;
    case 0x9: mod = 2; cod = 0; break;
    case 0xD: mod = 2; cod = 2; break;
    case 0x8: mod = 3; cod = 1; break;
    case 0xC: mod = 3; cod = 2; break;
    default: mod = 0; cod = 0;
  }
  int len = (int)((hb >> 5) & 0xFFF);
  if (len > 2048) len = 2048;
  const int plen = max(len - 4, 0);
  const int nc = mod == 0 ? 48 : mod == 1 ? 96 : mod == 2 ? 192 : 288;
  const int nd = cod == 0 ? nc / 2 : cod == 1 ? nc * 2 / 3 : nc * 3 / 4;
  const int nsym = (16 + 8 * plen + 32 + 6 + nd - 1) / nd;
  const uint32_t crc = crc32_wave(src + 3, plen, lane);
  uint32_t* dst = out + out_off[p];
  if (lane == 0) nsamp[p] = 640 + 160 * (1 + nsym);
  for (int i = lane; i < 640; i += 64) dst[i] = preamble[i];
  for (int i = lane; i < plen; i += 64) pay[i] = src[3 + i];
  __syncthreads();
  const Stream S{pay, plen, crc};
  uint8_t* cb = lds + lane * 288;
  for (int k = lane; k < 1 + nsym; k += 64) {
    s2 sub[48];
    if (k == 0) {                                          // SIGNAL: encode12 >>> BPSK
      uint32_t sr = 0;
      for (int i = 0; i < 24; i++) {
        const uint32_t b = (hb >> i) & 1u;
        cb[2 * i] = (uint8_t)((b ^ (sr >> 1) ^ (sr >> 2) ^ (sr >> 4) ^ (sr >> 5)) & 1u);
        cb[2 * i + 1] = (uint8_t)((b ^ sr ^ (sr >> 1) ^ (sr >> 2) ^ (sr >> 5)) & 1u);
        sr = ((sr << 1) | b) & 63u;
      }
#pragma unroll
      for (int i = 0; i < 48; i++) { uint8_t b[1] = {cb[kIntlv48[i]]}; sub[i] = map_bits<0>(b); }
    } else {
      const int fb = (k - 1) * nd;
      switch (mod) {
        case 0: symbol_bits<0>(S, fb, nd, cod, cb, sub); break;
        case 1: symbol_bits<1>(S, fb, nd, cod, cb, sub); break;
        case 2: symbol_bits<2>(S, fb, nd, cod, cb, sub); break;
        default: symbol_bits<3>(S, fb, nd, cod, cb, sub); break;
      }
    }
    // map_ofdm (map_ofdm.blk:63-107): carriers -32..31 of the 64-bin symbol go to bins
    // 96..127 and 0..31 of the 128-point IFFT (ifft.blk:41-43); pilots at 7, 21, 43, 57
    const int idx = k == 0 ? 127 : (k - 1) % 127;
    const short pv = ((kPilotNeg[idx >> 5] >> (idx & 31)) & 1u) ? (short)-10720 : (short)10720;
    s2 x[128];
#pragma unroll
    for (int i = 0; i < 128; i++) x[i] = (s2){0, 0};
#pragma unroll
    for (int i = 0; i < 48; i++) {
      const int c = data_bin(i);                            // carrier 1..26 or 38..63 (= -26..-1)
      x[c < 32 ? c : c + 64] = sub[i];
    }
    x[7] = (s2){pv, 0};
    x[21] = (s2){(short)-pv, 0};
    x[43 + 64] = (s2){pv, 0};
    x[57 + 64] = (s2){pv, 0};
    ifft128_inplace(x);
    uint32_t* o = dst + 640 + 160 * (int64_t)k;
#pragma unroll
    for (int t = 0; t < 128; t++) o[32 + t] = as_u32(x[bitrev7(t)]);
#pragma unroll
    for (int t = 0; t < 32; t++) o[t] = as_u32(x[bitrev7(96 + t)]);
  }
}

}  // namespace tx
}  // namespace zrx
