// FFTSafe<N> plans for every size __ext_sora_fft dispatches (csrc/sora_ext_lib.cpp:2672-2812):
// 16..2048 and the LTE sizes 12..1200.  Plain C++ (no HIP): the device kernel k_fft_n
// (zrx_fftn.hpp) and the host per-call path (zrx_host.cpp) execute the same plans.
//
// The reference recursion (FFTSSEEx<N>, csrc/fft_r4difx.hpp:99-218; FFTSSE_3W / FFTSSE_5W,
// csrc/sora_ext_lib_fft.hpp:111-430) applies one DIF stage to the whole block and recurses
// into its r sub-blocks; every sub-block at one depth has the same size, so the transform is
// a list of stages (radix r on sub-blocks of M), each a set of independent butterflies.
// A plan holds the stage list, the twiddles (round(32768 e^{-j2pi k n / M}) clamped to
// +-32767, the reference tables' formula) and the position of every output bin (the
// reference's bFFT{N}LUTMap, from the same recursion: a radix-4 stage leaves residues 0, 2,
// 1, 3 in its quarters, radix 3 / 5 in order, the base cases bit-reversed).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <vector>

namespace zrx {

constexpr int kFftMaxN = 2048;
constexpr int kFftMaxStages = 8;
constexpr int kFftSizes = 42;

struct FftStage {
  uint16_t radix;       // 3, 4, 5: a DIF stage; 0: the base case (4 or 8 points, M = 4 / 8)
  uint16_t M;           // sub-block size
  uint32_t tw;          // twiddle offset: entry (k - 1) * (M / radix) + n = tw<M, k>[n]
};
struct FftPlan {
  int32_t N, nst;
  FftStage st[kFftMaxStages];
  uint32_t pos;         // offset of N uint16: out[f] = x[pos[f]]
};

static const int kFftSizeList[kFftSizes] = {16, 32, 64, 128, 256, 512, 1024, 2048, 12, 24, 36, 48, 60, 72,
                                            96, 108, 120, 144, 180, 192, 216, 240, 288, 300, 324, 360, 384,
                                            432, 480, 540, 576, 600, 648, 720, 768, 864, 900, 960, 972, 1080,
                                            1152, 1200};

// FFTSSEEx<N> specialisations: radix 3 csrc/sora_ext_lib_fft.hpp:190-251, radix 5 :366-430,
// radix 4 otherwise, base cases 4 / 8 (csrc/fft_r4difx.hpp:111-218)
inline int fftn_radix(int N) {
  switch (N) {
    case 4: case 8: return 0;
    case 12: case 24: case 36: case 72: case 108: case 216: case 324: case 648: case 972: return 3;
    case 60: case 120: case 180: case 300: case 360: case 540: case 600: case 900: case 1080: return 5;
    default: return 4;
  }
}
inline void fftn_freq(int N, int* idx) {
  const int r = fftn_radix(N);
  if (r == 0) {
    for (int p = 0; p < N; p++) idx[p] = N == 4 ? ((p & 1) << 1 | (p >> 1)) : ((p & 1) << 2 | (p & 2) | (p >> 2));
    return;
  }
  const int M = N / r;
  std::vector<int> sub(M);
  fftn_freq(M, sub.data());
  static const int res4[4] = {0, 2, 1, 3};
  for (int q = 0; q < r; q++)
    for (int p = 0; p < M; p++) idx[q * M + p] = r * sub[p] + (r == 4 ? res4[q] : q);
}
// twFFTLUT{M}_{k}[n] (csrc/sora_ext_lib_fft_coeffs.hpp): round(32768 e^{-j 2 pi k n / M}),
// each part clamped to +-32767 (the oracle's zo_twiddle, checked against the brick)
inline uint32_t fftn_twiddle(int M, int k, int n) {
  const double ang = -2.0 * M_PI * (double)k * (double)n / (double)M;
  double r = std::floor(32768.0 * std::cos(ang) + 0.5), i = std::floor(32768.0 * std::sin(ang) + 0.5);
  r = std::min(32767.0, std::max(-32767.0, r));
  i = std::min(32767.0, std::max(-32767.0, i));
  return (uint32_t)(uint16_t)(int16_t)r | ((uint32_t)(uint16_t)(int16_t)i << 16);
}
inline int fftn_index(int N) {
  for (int i = 0; i < kFftSizes; i++)
    if (kFftSizeList[i] == N) return i;
  return -1;
}

struct FftPlans {
  std::vector<FftPlan> plans;     // kFftSizes, in kFftSizeList order
  std::vector<uint32_t> tw;       // complex16 twiddles (re | im << 16)
  std::vector<uint16_t> pos;
};
inline FftPlans fftn_build_plans() {
  FftPlans R;
  R.plans.resize(kFftSizes);
  for (int i = 0; i < kFftSizes; i++) {
    const int N = kFftSizeList[i];
    FftPlan& P = R.plans[i];
    P.N = N; P.nst = 0;
    for (int M = N;;) {
      const int r = fftn_radix(M);
      FftStage& st = P.st[P.nst++];
      st.radix = (uint16_t)r; st.M = (uint16_t)M; st.tw = (uint32_t)R.tw.size();
      if (r == 0) break;
      for (int k = 1; k < r; k++)
        for (int n = 0; n < M / r; n++) R.tw.push_back(fftn_twiddle(M, k, n));
      M /= r;
    }
    std::vector<int> idx(N);
    fftn_freq(N, idx.data());
    P.pos = (uint32_t)R.pos.size();
    R.pos.resize(R.pos.size() + N);
    for (int p = 0; p < N; p++) R.pos[P.pos + idx[p]] = (uint16_t)p;
  }
  return R;
}

}  // namespace zrx
