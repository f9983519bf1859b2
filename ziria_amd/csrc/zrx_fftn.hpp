// FFTSafe<N> for every size __ext_sora_fft dispatches (csrc/sora_ext_lib.cpp:2672-2812):
// 16..2048 and the LTE sizes 12..1200, one workgroup per transform, the N values in LDS.
//
// The plans (stage list, twiddles, output positions) come from zrx_fftplan.hpp; each stage's
// butterflies are independent, so the workgroup's threads share them between two barriers.
// Per butterfly the integer semantics are the SSE bricks' (saturating int16 adds, madd-wrap
// mul_shift, XOR-as-negate), so the result is bit-exact.
#pragma once
#include "zrx_device.hpp"
#include "zrx_fftplan.hpp"

namespace zrx {

// FFTSSEEx<8> (csrc/fft_r4difx.hpp:142-218) per complex value: input >> 3; d = x[k] -
// x[k+4], s = x[k] + x[k+4]; the lower half rotates d2, d3 by (im, ~re), pairs them with d0,
// d1, multiplies by (32767,0), (23169,-23169), (32767,0), (-23169,-23169) and finishes with
// XOR-as-negate pairs; the upper half is the 4-point DFT of s with the same pairing.
__device__ __forceinline__ void fft8(s2* x) {
  s2 d[4], s[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const s2 a = x[k] >> (s2){3, 3}, b = x[k + 4] >> (s2){3, 3};
    d[k] = sat_sub(a, b);
    s[k] = sat_add(a, b);
  }
  const s2 m2 = {d[2].y, (short)~d[2].x}, m3 = {d[3].y, (short)~d[3].x};
  const s2 f0 = mul_shift(sat_add(d[0], m2), 32767, 0), f1 = mul_shift(sat_add(d[1], m3), 23169, -23169);
  const s2 f2 = mul_shift(sat_add(~m2, d[0]), 32767, 0), f3 = mul_shift(sat_add(~m3, d[1]), -23169, -23169);
  const s2 t0 = sat_add(s[0], s[2]), t1 = sat_add(s[1], s[3]), t2 = sat_add(~s[2], s[0]);
  const s2 t3a = sat_add(~s[3], s[1]);
  const s2 t3 = {t3a.y, (short)~t3a.x};
  x[0] = sat_add(t0, t1);
  x[1] = sat_add(~t1, t0);
  x[2] = sat_add(t2, t3);
  x[3] = sat_add(~t3, t2);
  x[4] = sat_add(f0, f1);
  x[5] = sat_add(f0, ~f1);
  x[6] = sat_add(f2, f3);
  x[7] = sat_add(f2, ~f3);
}

__device__ __forceinline__ s2 mul_tw(s2 a, uint32_t t) { const s2 w = as_s2(t); return mul_shift(a, w.x, w.y); }

// One butterfly of a stage: radix r over x[base + q m], twiddle index n.
__device__ __forceinline__ void fftn_butterfly(uint32_t* x, int radix, int base, int m, int n, const uint32_t* tw) {
  if (radix == 4) {                                    // FFTSSE<M> (csrc/fft_r4difx.hpp:54-97)
    const s2 a = shr2(as_s2(x[base])), b = shr2(as_s2(x[base + m])), c = shr2(as_s2(x[base + 2 * m])),
             d = shr2(as_s2(x[base + 3 * m]));
    const s2 ac = sat_add(a, c), bd = sat_add(b, d), a_c = sat_sub(a, c), b_d = sat_sub(b, d);
    const s2 jb = mul_j(b_d);
    x[base] = as_u32(sat_add(ac, bd));
    x[base + m] = as_u32(mul_tw(sat_sub(ac, bd), tw[m + n]));
    x[base + 2 * m] = as_u32(mul_tw(sat_sub(a_c, jb), tw[n]));
    x[base + 3 * m] = as_u32(mul_tw(sat_add(a_c, jb), tw[2 * m + n]));
  } else if (radix == 3) {                             // FFTSSE_3<M> (csrc/sora_ext_lib_fft.hpp:111-171)
    const s2 a = shr2(as_s2(x[base])), b = shr2(as_s2(x[base + m])), c = shr2(as_s2(x[base + 2 * m]));
    const s2 bk1 = mul_shift(b, -16384, -28378), bk2 = mul_shift(b, -16384, 28378);
    const s2 ck1 = mul_shift(c, -16384, -28378), ck2 = mul_shift(c, -16384, 28378);
    x[base] = as_u32(sat_add(sat_add(a, b), c));
    x[base + m] = as_u32(mul_tw(sat_add(sat_add(a, bk1), ck2), tw[n]));
    x[base + 2 * m] = as_u32(mul_tw(sat_add(sat_add(a, bk2), ck1), tw[m + n]));
  } else if (radix == 5) {                             // FFTSSE_5<M> (csrc/sora_ext_lib_fft.hpp:253-349)
    const s2 sh = {3, 3};
    const s2 a = as_s2(x[base]) >> sh, b = as_s2(x[base + m]) >> sh, c = as_s2(x[base + 2 * m]) >> sh,
             d = as_s2(x[base + 3 * m]) >> sh, e = as_s2(x[base + 4 * m]) >> sh;
    auto k1 = [](s2 v) { return mul_shift(v, 10126, -31164); };
    auto k2 = [](s2 v) { return mul_shift(v, -26510, -19261); };
    auto k3 = [](s2 v) { return mul_shift(v, -26510, 19261); };
    auto k4 = [](s2 v) { return mul_shift(v, 10126, 31164); };
    x[base] = as_u32(sat_add(sat_add(sat_add(a, b), sat_add(c, d)), e));
    x[base + m] = as_u32(mul_tw(sat_add(sat_add(sat_add(a, k1(b)), sat_add(k2(c), k3(d))), k4(e)), tw[n]));
    x[base + 2 * m] = as_u32(mul_tw(sat_add(sat_add(sat_add(a, k2(b)), sat_add(k4(c), k1(d))), k3(e)), tw[m + n]));
    x[base + 3 * m] = as_u32(mul_tw(sat_add(sat_add(sat_add(a, k3(b)), sat_add(k1(c), k4(d))), k2(e)), tw[2 * m + n]));
    x[base + 4 * m] = as_u32(mul_tw(sat_add(sat_add(sat_add(a, k4(b)), sat_add(k3(c), k2(d))), k1(e)), tw[3 * m + n]));
  }
}

// count transforms of plan->N points: in/out are N complex16 each (may alias); one
// workgroup of 256 threads per transform (block-stride over count).
__global__ __launch_bounds__(256) void k_fft_n(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                               int64_t count, const FftPlan* __restrict__ plan,
                                               const uint32_t* __restrict__ twp, const uint16_t* __restrict__ posp) {
  __shared__ uint32_t x[kFftMaxN];
  const int N = plan->N, nst = plan->nst;
  const int t = threadIdx.x;
  const uint16_t* pos = posp + plan->pos;
  for (int64_t b = blockIdx.x; b < count; b += gridDim.x) {
    const uint32_t* src = in + b * N;
    for (int i = t; i < N; i += 256) x[i] = src[i];
    __syncthreads();
    for (int s = 0; s < nst; s++) {
      const FftStage st = plan->st[s];
      if (st.radix == 0) {                             // base cases FFTSSEEx<4> / <8>
        for (int blk = t; blk < N / st.M; blk += 256) {
          s2 v[8];
          for (int i = 0; i < st.M; i++) v[i] = as_s2(x[blk * st.M + i]);
          if (st.M == 4) fft4(v); else fft8(v);
          for (int i = 0; i < st.M; i++) x[blk * st.M + i] = as_u32(v[i]);
        }
      } else {
        const int m = st.M / st.radix;
        for (int bf = t; bf < N / st.radix; bf += 256) {
          const int blk = bf / m, n = bf - blk * m;
          fftn_butterfly(x, st.radix, blk * st.M + n, m, n, twp + st.tw);
        }
      }
      __syncthreads();
    }
    uint32_t* dst = out + b * N;
    for (int f = t; f < N; f += 256) dst[f] = x[pos[f]];
    __syncthreads();                                   // x is reloaded by the next transform
  }
}

}  // namespace zrx
