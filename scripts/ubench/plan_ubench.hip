// k_pkt_plan alone on config-3 / config-5 / config-2 shaped vparams, HIP-event timed; built
// with -DZRX_PLAN_CUT=N to stop after phase N (1 scans, 2 + column total, 3 + key count,
// 5 + scatter, 99 all).  usage: plan_ubench (prints one line per shape)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../ziria_amd/csrc/zrx_kernels.hip"
using namespace zrx;

static int g_split = 0;   // argv[1] = 1: k_pkt_plan as the rx chain launches it (mixed rows left to k_pkt_rows)
static void run(const char* name, const std::vector<int32_t>& vp, int npkts, bool chain) {
  int32_t *d_vp, *d_nrows, *d_order, *d_bits, *d_dsym, *d_w;
  int64_t* d_off;
  int2* d_rows;
  uint8_t* d_segs;
  hipMalloc(&d_vp, vp.size() * 4);
  hipMemcpy(d_vp, vp.data(), vp.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&d_nrows, 32); hipMalloc(&d_order, npkts * 4); hipMalloc(&d_bits, npkts * 4);
  hipMalloc(&d_dsym, npkts * 4 + 8); hipMalloc(&d_w, (size_t)npkts * 1400 / 64 * 4 + 64);
  hipMalloc(&d_off, npkts * 8); hipMalloc(&d_rows, (size_t)(npkts + 16384) * 8); hipMalloc(&d_segs, npkts);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  auto launch = [&]() {
    k_pkt_plan<<<1, 1024>>>(d_vp, npkts, chain ? d_off : nullptr, d_dsym, d_w, d_rows, d_nrows, d_segs, d_order, d_bits, 256, npkts + 16384, g_split, nullptr);
  };
  for (int i = 0; i < 5; i++) launch();
  hipEventRecord(a);
  for (int i = 0; i < 50; i++) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  int nr[2];
  hipMemcpy(nr, d_nrows, 8, hipMemcpyDeviceToHost);
  std::printf("split %d cut %d %-8s %6d pkts: %7.2f us  rows %d\n", g_split, ZRX_PLAN_CUT, name, npkts, ms * 1000 / 50, nr[0]);
}

int main(int argc, char** argv) {
  g_split = argc > 1 ? std::atoi(argv[1]) : 0;
  const int n = 16384;
  std::vector<int32_t> c3(4 * n), c5(4 * n), c2(4 * 4096);
  for (int i = 0; i < n; i++) { c3[4 * i] = 1506; c3[4 * i + 1] = 2; c3[4 * i + 2] = 56 * 288; c3[4 * i + 3] = 3; }
  srand(5);
  const int nd[4] = {48, 96, 192, 288}, cod[8] = {0, 2, 0, 2, 0, 2, 1, 2}, mods[8] = {0, 0, 1, 1, 2, 2, 3, 3};
  for (int i = 0; i < n; i++) {
    const int m = rand() % 8, len = 64 + rand() % 4032, mod = mods[m], cr = cod[m];
    const int ncb = nd[mod], ndb = cr == 0 ? ncb / 2 : cr == 1 ? ncb * 2 / 3 : ncb * 3 / 4;
    const int ok = len <= 2048, need = (16 + 8 * (len + 2) + 6 + ndb - 1) / ndb;
    c5[4 * i] = ok ? len + 2 : 2050; c5[4 * i + 1] = cr; c5[4 * i + 2] = ok ? need * ncb : 0; c5[4 * i + 3] = mod;
  }
  for (int i = 0; i < 4096; i++) { c2[4 * i] = 1500; c2[4 * i + 1] = 0; c2[4 * i + 2] = 24048; c2[4 * i + 3] = 0; }
  run("config3", c3, n, true);
  run("config5", c5, n, true);
  run("config2", c2, 4096, false);
  return 0;
}
