// Probe: how far from the PilotTrack rotation table (rint(32767 cos/sin(2 r pi' / 65536)),
// pi' = 3.141593, zrx_api.hip make_trig_tables) are fp32 evaluations on gfx950?  For every
// r in 0..65535 the device computes 32767 cos / sin in fp32 (hardware v_cos/v_sin on the angle
// in revolutions, and the OCML cosf/sinf), the host compares with the double-precision value.
// Prints the max abs error (table units) and how many r would fall in an ambiguity band of
// +-eps around .5 for a few eps.
// build: hipcc --offload-arch=gfx950 -O3 -o trig_probe trig_probe.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k_probe(float* out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= 65536) return;
  // revolutions: r / 65536 * pi' / pi, as r * 2^-16 (exact) + r * 2^-16 * (pi'/pi - 1)
  const float t0 = (float)r * (1.0f / 65536.0f);
  const float corr = (float)(1.1026579e-7);   // pi'/pi - 1 (3.141593 / 3.14159265358979 - 1)
  const float t = __builtin_fmaf(t0, corr, t0);
  out[4 * r + 0] = 32767.0f * __builtin_amdgcn_cosf(t);
  out[4 * r + 1] = 32767.0f * __builtin_amdgcn_sinf(t);
  const float th = (float)r * (float)(2.0 * 3.141593 / 65536.0);
  out[4 * r + 2] = 32767.0f * cosf(th);
  out[4 * r + 3] = 32767.0f * sinf(th);
}

int main() {
  float* d;
  hipMalloc(&d, 65536 * 16);
  k_probe<<<256, 256>>>(d);
  std::vector<float> h(65536 * 4);
  hipMemcpy(h.data(), d, 65536 * 16, hipMemcpyDeviceToHost);
  const double pi = 3.141593;
  const char* names[4] = {"hw_cos", "hw_sin", "ocml_cos", "ocml_sin"};
  const double eps[5] = {0.002, 0.005, 0.01, 0.02, 0.05};
  for (int v = 0; v < 4; v++) {
    double maxerr = 0;
    int mism = 0, amb[5] = {0, 0, 0, 0, 0}, bad[5] = {0, 0, 0, 0, 0};
    for (int r = 0; r < 65536; r++) {
      const double ang = (double)r * 2.0 * pi / 65536.0;
      const double ex = 32767.0 * ((v & 1) ? std::sin(ang) : std::cos(ang));
      const double tab = std::nearbyint(ex);
      const double got = h[4 * r + v];
      maxerr = std::fmax(maxerr, std::fabs(got - ex));
      if (std::nearbyint(got) != tab) mism++;
      const double fr = std::fabs(got - std::nearbyint(got));   // distance to the nearest integer
      for (int e = 0; e < 5; e++) {
        if (fr > 0.5 - eps[e]) amb[e]++;
        else if (std::nearbyint(got) != tab) bad[e]++;
      }
    }
    printf("%-9s maxerr %.5f  mismatches %d", names[v], maxerr, mism);
    for (int e = 0; e < 5; e++) printf("  eps %.3f: amb %d bad %d", eps[e], amb[e], bad[e]);
    printf("\n");
  }
  return 0;
}
