// RX front end: receiver() of code/WiFi/receiver/receiver.blk:57-72
// up to the data symbols, batched over independent captures (one receiver() per capture).
//
//   k_fe_detect  one wave per capture: downSample (downSample.blk:31-57, odd samples) ->
//                removeDC (removeDC.blk:25-85) -> cca (cca/cca_tufv.blk:103-338) in 16-sample
//                blocks; lane i < 16 holds sample i of the block and correlates the STS
//                pattern at shift i (its 16 pattern values and 9-deep history in registers)
//   k_fe_lts     one lane per capture: LTS (OFDM/LTS.blk:113-203): AGC shift, FFT of both
//                long training symbols, calcCoeff, sum -> the 64 channel coefficients
//   k_fe_gather  one wave per capture: DataSymbol (OFDM/DataSymbol.blk:24-30), 64 of every
//                80 samples from the capture into the symbol layout of the decode chain
// The decode chain then runs with ChannelEqualization + PilotTrack (rx_chain with chan).
#pragma once
#include "zrx_device.hpp"

namespace zrx {
namespace fe {

constexpr int kDetWords = 8;    // det[8p..] = {detected, noSamples, shift, energy, noise, maxCorr, consumed, data_start}

__device__ __forceinline__ uint32_t ld_sample(const uint32_t* __restrict__ s, int64_t base, int j, int ds) {
  return s[base + (ds ? 2 * (int64_t)j + 1 : (int64_t)j)];    // permutatew1313 + interleave_loww
}
__device__ __forceinline__ s2 sra(s2 v, int k) { return v >> (s2){(short)k, (short)k}; }
__device__ __forceinline__ int lo16(uint32_t w) { return (int)(short)(w & 0xFFFFu); }
__device__ __forceinline__ int hi16(uint32_t w) { return (int)(short)(w >> 16); }

// 16-lane sum (lanes 0..15 of the wave), wrapping uint32, result in every lane of row 0
__device__ __forceinline__ uint32_t row_sum(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
  return v;
}

__global__ __launch_bounds__(256) void k_fe_detect(const uint32_t* __restrict__ samples, const int64_t* __restrict__ cap_off,
                                                   const int32_t* __restrict__ cap_len, int ncap, int downsample,
                                                   int32_t thr, const uint32_t* __restrict__ pattern,
                                                   int32_t* __restrict__ det) {
  const int lane = threadIdx.x & 63;
  const int p = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (p >= ncap) return;
  const int64_t base = cap_off[p];
  const int len_in = cap_len[p];
  const int n = downsample ? (len_in / 8) * 4 : len_in;        // samples of the receiver's stream
  const int ci = lane & 15;                                     // correlation shift of this lane
  s2 pat[16];
#pragma unroll
  for (int j = 0; j < 16; j++) pat[j] = as_s2(pattern[ci * 16 + j]);
  uint32_t mre = 0, mim = 0;                                    // mul_hist[ci]
  uint32_t hist[9];
#pragma unroll
  for (int k = 0; k < 9; k++) hist[k] = 0;
  int dc_re = 0, dc_im = 0, sum_re = 0, sum_im = 0, cnt = 8;   // removeDC state (dc[0..3] are equal)
  int idle = 0, idle_cnt = 0, iterind = 0, noInc = 0, maxInd = 0, oldInd = 0, oldOldInd = 0;
  int32_t oldOldCorr = 0, oldCorr = 0, maxCorr = 0, iEnergy = 0, iNoise = 0;
  int pos = 0, detected = 0;
  while (!detected && pos + 16 <= n) {
    const s2 x = lane < 16 ? as_s2(ld_sample(samples, base, pos + lane, downsample)) : (s2){0, 0};
    pos += 16;
    // removeDC: 4 steps of 4 samples; dc updates after the step in which cnt reaches 0
    s2 y = {0, 0};
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const s2 yy = x - (s2){(short)dc_re, (short)dc_im};       // v_sub_complex16 (wrapping)
      if ((lane >> 2) == s) y = yy;
      const uint32_t t = as_u32(sra(yy, 5));
      const uint32_t t0 = __builtin_amdgcn_readlane(t, 4 * s), t1 = __builtin_amdgcn_readlane(t, 4 * s + 1);
      const uint32_t t2 = __builtin_amdgcn_readlane(t, 4 * s + 2), t3 = __builtin_amdgcn_readlane(t, 4 * s + 3);
      sum_re = (short)(sum_re + (short)(lo16(t0) + lo16(t1) + lo16(t2) + lo16(t3)));   // v_hadd (num16), v_add
      sum_im = (short)(sum_im + (short)(hi16(t0) + hi16(t1) + hi16(t2) + hi16(t3)));
      if (cnt == 0) {
        dc_re = (short)(dc_re + (sum_re >> 2));
        dc_im = (short)(dc_im + (sum_im >> 2));
        cnt = 8;
        sum_re = sum_im = 0;
      }
      cnt--;
    }
    // calcEnergy: |y >> 4|^2 summed over the block (madd, wrapping int32 sum)
    const s2 e4 = sra(sra(y, 2), 2);
    const uint32_t e = lane < 16 ? (uint32_t)__builtin_amdgcn_sdot2(e4, e4, 0, false) : 0u;
    iEnergy = (int32_t)__builtin_amdgcn_readlane(row_sum(e), 0);
    if (!idle) {                                                 // until initial_idle (:160-179)
      if (iEnergy < thr) idle_cnt++; else idle_cnt = 0;
      if (idle_cnt >= 20) { idle = 1; iNoise = iEnergy; iterind = 0; }
      iterind++;
      continue;
    }
    // v_correlate(pattern[ci], input): sum of pattern * conj(input), input = y >> 7
    const uint32_t in = as_u32(sra(y, 7));
    uint32_t cre = 0, cim = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const s2 v = as_s2(__builtin_amdgcn_readlane(in, j));
      cre += (uint32_t)__builtin_amdgcn_sdot2(v, pat[j], 0, false);
      cim += (uint32_t)__builtin_amdgcn_sdot2((s2){(short)-v.y, v.x}, pat[j], 0, false);
    }
    // corrc * conj_complex32(mul_hist) (complex32_mult, csrc/numerics.c:107-113), |re| + |im|
    const uint32_t hre = mre, him = 0u - mim;
    const uint32_t pre_ = cre * hre - cim * him, pim = cim * hre + cre * him;
    const uint32_t are = (int32_t)pre_ >= 0 ? pre_ : 0u - pre_, aim = (int32_t)pim >= 0 ? pim : 0u - pim;
    mre = cre; mim = cim;
    uint32_t corr = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) { hist[k] = hist[k + 1]; corr += hist[k]; }
    hist[8] = are + aim;
    corr += hist[8];
    // first shift with corr > running max (strict), starting from 0
    int32_t mc = 0;
    int mi = -1;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const int32_t c = (int32_t)__builtin_amdgcn_readlane(corr, k);
      if (c > mc) { mc = c; mi = k; }
    }
    maxCorr = mc;
    if (mi >= 0) maxInd = mi;
    const int32_t norm = iEnergy == 0 ? 0 : maxCorr / iEnergy;
    if (iEnergy > thr && noInc > 4 && (oldCorr > maxCorr || oldInd != maxInd) && norm > 96) detected = 1;
    if (oldOldCorr < oldCorr && oldCorr < maxCorr && oldOldInd == oldInd && oldInd == maxInd) noInc++;
    else noInc = 0;
    oldOldCorr = oldCorr; oldCorr = maxCorr;
    oldOldInd = oldInd; oldInd = maxInd;
    iterind++;
  }
  if (lane == 0) {
    int32_t* d = det + (int64_t)p * kDetWords;
    d[0] = detected; d[1] = 16 * iterind + oldInd; d[2] = oldInd; d[3] = iEnergy; d[4] = iNoise;
    d[5] = maxCorr; d[6] = pos; d[7] = pos + 144;
  }
}

// calcCoeff (LTS.blk:71-111) of one FFT output x (bin b at x[bitrev6(b)]) into c[64]
__device__ __forceinline__ void calc_coeff(const s2* x, uint32_t* __restrict__ c, bool accumulate) {
#pragma unroll
  for (int b = 0; b < 64; b++) {
    uint32_t w = 0;
    if (b < 28 || b >= 36) {
      const s2 f = x[bitrev6(b)];
      const int32_t sq = __builtin_amdgcn_sdot2(f, f, 0, false) >> 6;      // v_shift_right_int32
      const int L = ((kLts11aBits >> b) & 1ull) ? 1600 : -1600;            // aLTSSeq11a (:40-55)
      const int32_t re = (int32_t)((uint32_t)f.x * (uint32_t)L);          // x * conj(y), x = LTS (im 0)
      const int32_t im = (int32_t)((uint32_t)(int)(short)-f.y * (uint32_t)L);
      if (sq > 1) w = (uint32_t)(uint16_t)(short)(re / sq) | ((uint32_t)(uint16_t)(short)(im / sq) << 16);
    }
    if (accumulate) {                                                       // v_add_complex16 (wrapping)
      const uint32_t o = c[b];
      w = (uint32_t)(uint16_t)(short)(lo16(o) + lo16(w)) | ((uint32_t)(uint16_t)(short)(hi16(o) + hi16(w)) << 16);
    }
    c[b] = w;
  }
}
__device__ __forceinline__ s2 shift_c16(s2 v, int sh) {           // v_shift_left / right_complex16
  if (sh > 0) return (s2){(short)(sh > 15 ? 0 : (uint16_t)((uint16_t)v.x << sh)), (short)(sh > 15 ? 0 : (uint16_t)((uint16_t)v.y << sh))};
  const int r = -sh > 15 ? 15 : -sh;
  return sra(v, r);
}

// agc_shift = round_int32(log2(1000 / sqrt(amp))) (LTS.blk:146, csrc/ext_math.c:70-80) in fp64;
// the amplitudes where the value is an exact .5 tie take the host's (reference libm) value.
struct AgcTies { int32_t amp[8]; int32_t agc[8]; };
__device__ __forceinline__ int agc_shift(int32_t amp, const AgcTies& T) {
#pragma unroll
  for (int i = 0; i < 8; i++)
    if (amp == T.amp[i]) return T.agc[i];
  const double d = log(1000.0 / sqrt((double)amp)) / log(2.0);
  return (int)((d > 0) ? (d + 0.5) : (d - 0.5));
}

__global__ __launch_bounds__(64) void k_fe_lts(const uint32_t* __restrict__ samples, const int64_t* __restrict__ cap_off,
                                               const int32_t* __restrict__ cap_len, int ncap, int downsample,
                                               const int32_t* __restrict__ det, AgcTies ties,
                                               uint32_t* __restrict__ chan) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ncap) return;
  const int32_t* d = det + (int64_t)p * kDetWords;
  const int n = downsample ? (cap_len[p] / 8) * 4 : cap_len[p];
  uint32_t* c = chan + (int64_t)p * 64;
  if (!d[0] || d[6] + 144 > n) {
    for (int b = 0; b < 64; b++) c[b] = 0;
    return;
  }
  const int64_t base = cap_off[p];
  const int shift = d[2], start = d[6];
  const int agc = agc_shift(d[5], ties);
#pragma unroll
  for (int half = 0; half < 2; half++) {                 // preamble xp[16-shift..], delayed xp[80-shift..]
    s2 x[64];
    const int o = start + (half ? 80 : 16) - shift;
#pragma unroll
    for (int j = 0; j < 64; j++) x[j] = shift_c16(as_s2(ld_sample(samples, base, o + j, downsample)), agc);
    fft64_inplace(x);
    calc_coeff(x, c, half == 1);
  }
  const int agcs = agc - 1;
  for (int b = 0; b < 64; b++) c[b] = as_u32(shift_c16(as_s2(c[b]), agcs));
}

// DataSymbol: symbol k of capture p = stream samples [data_start + 80k + 16 - shift, +64)
__global__ __launch_bounds__(256) void k_fe_gather(const uint32_t* __restrict__ samples, const int64_t* __restrict__ cap_off,
                                                   const int32_t* __restrict__ cap_len, int ncap, int downsample,
                                                   const int32_t* __restrict__ det, int max_sym,
                                                   uint32_t* __restrict__ sym, int64_t* __restrict__ sym_off,
                                                   int32_t* __restrict__ nsym) {
  const int lane = threadIdx.x & 63;
  const int p = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (p >= ncap) return;
  const int32_t* d = det + (int64_t)p * kDetWords;
  const int n = downsample ? (cap_len[p] / 8) * 4 : cap_len[p];
  const int d0 = d[7];
  const int ns = d[0] && d0 <= n ? min((n - d0) / 80, max_sym) : 0;
  if (lane == 0) { sym_off[p] = (int64_t)p * max_sym; nsym[p] = ns; }
  const int64_t base = cap_off[p];
  uint32_t* dst = sym + (int64_t)p * max_sym * 64;
  for (int k = 0; k < ns; k++)
    dst[(int64_t)k * 64 + lane] = ld_sample(samples, base, d0 + 80 * k + 16 - d[2] + lane, downsample);
}

}  // namespace fe
}  // namespace zrx
