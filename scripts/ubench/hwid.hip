// Where does the dispatcher put the blocks of a k_viterbi3-shaped launch (256 threads,
// ~39 KB LDS, 4 blocks per CU)?  Each wave records HW_REG_HW_ID and HW_REG_XCC_ID; the
// host prints, per block, the (xcc, se, sh, cu) of wave 0 and the SIMD ids of its 4 waves,
// and how many blocks share each CU among the first N.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

__global__ __launch_bounds__(256, 4) void probe(uint32_t* out, int spin) {
  __shared__ uint8_t lds[39 * 1024];
  lds[threadIdx.x] = (uint8_t)threadIdx.x;
  const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
  const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);
  uint32_t acc = lds[(threadIdx.x * 7) & 255];
  for (int i = 0; i < spin; i++) acc = acc * 1664525u + 1013904223u;
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    out[2 * w] = hw;
    out[2 * w + 1] = xcc | (acc & 0x80000000u);
  }
}

int main() {
  const int nb = 1024;
  uint32_t* d;
  hipMalloc(&d, nb * 4 * 2 * 4);
  probe<<<nb, 256>>>(d, 200000);
  hipDeviceSynchronize();
  std::vector<uint32_t> h(nb * 8);
  hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  std::map<uint32_t, int> cu_count;
  for (int b = 0; b < nb; b++) {
    const uint32_t hw = h[8 * b], xcc = h[8 * b + 1] & 0xF;
    const uint32_t se = (hw >> 13) & 7, sh = (hw >> 12) & 1, cu = (hw >> 8) & 15;
    const uint32_t key = (xcc << 12) | (se << 8) | (sh << 4) | cu;
    cu_count[key]++;
    if (b < 80 || (b >= 256 && b < 290))
      printf("block %4d xcc %u se %u sh %u cu %2u simd %u %u %u %u wave %u %u %u %u\n", b, xcc, se, sh, cu,
             (h[8 * b] >> 4) & 3, (h[8 * b + 2] >> 4) & 3, (h[8 * b + 4] >> 4) & 3, (h[8 * b + 6] >> 4) & 3,
             h[8 * b] & 15, h[8 * b + 2] & 15, h[8 * b + 4] & 15, h[8 * b + 6] & 15);
  }
  std::map<int, int> hist;
  for (auto& kv : cu_count) hist[kv.second]++;
  printf("distinct CUs %zu;", cu_count.size());
  for (auto& kv : hist) printf(" %d CUs with %d blocks;", kv.second, kv.first);
  printf("\n");
  // first 256 blocks: how many distinct CUs
  std::map<uint32_t, int> first;
  for (int b = 0; b < 256; b++) {
    const uint32_t hw = h[8 * b], xcc = h[8 * b + 1] & 0xF;
    first[(xcc << 12) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)]++;
  }
  std::map<int, int> fh;
  for (auto& kv : first) fh[kv.second]++;
  printf("first 256 blocks: %zu distinct CUs;", first.size());
  for (auto& kv : fh) printf(" %d CUs with %d;", kv.second, kv.first);
  printf("\n");
  return 0;
}
