// Does the order of fast (VOP2 v_add_u32, ~2.7 cycles) and slow (VOP3P v_pk_min_u16, ~4.8
// cycles) VALU instructions change their mixed cost?  16 independent registers per wave;
// each kernel issues 8 adds and 8 pk_mins per iteration in a given order.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096
#define A(i) "v_add_u32 %[r" #i "], %[c], %[r" #i "]\n\t"
#define M(i) "v_pk_min_u16 %[r" #i "], %[c], %[r" #i "]\n\t"
#define P(i) "v_perm_b32 %[r" #i "], %[c], %[r" #i "], %[c]\n\t"
#define D(i) "v_add_u32_dpp %[r" #i "], %[c], %[r" #i "] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
#define S(i) "v_sub_u32 %[r" #i "], %[c], %[r" #i "]\n\t"

#define DEFK(NAME, BODY)                                                                   \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t s) {                 \
    uint32_t r0 = threadIdx.x, r1 = r0 ^ 1, r2 = r0 ^ 2, r3 = r0 ^ 3, r4 = r0 + 4, r5 = r0 + 5, \
             r6 = r0 + 6, r7 = r0 + 7, r8 = r0 + 8, r9 = r0 + 9, r10 = r0 + 10, r11 = r0 + 11, \
             r12 = r0 + 12, r13 = r0 + 13, r14 = r0 + 14, r15 = r0 + 15, c = s * 3u + threadIdx.x; \
    for (int it = 0; it < ITERS; it++) {                                                   \
      asm volatile(BODY : [r0] "+v"(r0), [c] "+v"(c), [r1] "+v"(r1), [r2] "+v"(r2), [r3] "+v"(r3),  \
                   [r4] "+v"(r4), [r5] "+v"(r5), [r6] "+v"(r6), [r7] "+v"(r7), [r8] "+v"(r8), \
                   [r9] "+v"(r9), [r10] "+v"(r10), [r11] "+v"(r11), [r12] "+v"(r12),       \
                   [r13] "+v"(r13), [r14] "+v"(r14), [r15] "+v"(r15)                        \
                   : [s] "s"(s) : "memory");                                               \
    }                                                                                      \
    out[blockIdx.x * 256 + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7 ^ r8 ^ r9 ^ r10 ^ \
        r11 ^ r12 ^ r13 ^ r14 ^ r15;                                                       \
  }

// 16 adds / 16 pk_mins alone
DEFK(k_a16, A(0) A(1) A(2) A(3) A(4) A(5) A(6) A(7) A(8) A(9) A(10) A(11) A(12) A(13) A(14) A(15))
DEFK(k_m16, M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15))
// 8 + 8 interleaved one by one (independent registers)
DEFK(k_am1, A(0) M(1) A(2) M(3) A(4) M(5) A(6) M(7) A(8) M(9) A(10) M(11) A(12) M(13) A(14) M(15))
// 8 + 8 in two runs
DEFK(k_am8, A(0) A(2) A(4) A(6) A(8) A(10) A(12) A(14) M(1) M(3) M(5) M(7) M(9) M(11) M(13) M(15))
// runs of 4
DEFK(k_am4, A(0) A(2) A(4) A(6) M(1) M(3) M(5) M(7) A(8) A(10) A(12) A(14) M(9) M(11) M(13) M(15))
// runs of 2
DEFK(k_am2, A(0) A(2) M(1) M(3) A(4) A(6) M(5) M(7) A(8) A(10) M(9) M(11) A(12) A(14) M(13) M(15))
// dependent pairs: add then pk_min on the same register (the ACS shape), interleaved over regs
DEFK(k_dep1, A(0) M(0) A(1) M(1) A(2) M(2) A(3) M(3) A(4) M(4) A(5) M(5) A(6) M(6) A(7) M(7))
DEFK(k_dep4, A(0) A(1) A(2) A(3) M(0) M(1) M(2) M(3) A(4) A(5) A(6) A(7) M(4) M(5) M(6) M(7))
// the body's mix per dword-column: 2 adds (one DPP), 1 pk_min, 0.75 sub, 0.67 perm
DEFK(k_mixa, P(0) S(1) A(2) D(3) M(4) P(5) S(6) A(7) D(8) M(9) A(10) S(11) A(12) M(13) A(14) M(15))
DEFK(k_mixb, A(2) A(7) A(10) A(12) A(14) S(1) S(6) S(11) P(0) P(5) D(3) D(8) M(4) M(9) M(13) M(15))
DEFK(k_mixc, P(0) P(5) D(3) D(8) M(4) M(9) M(13) M(15) A(2) A(7) A(10) A(12) A(14) S(1) S(6) S(11))

typedef void (*KF)(uint32_t*, uint32_t);
int main() {
  struct { const char* n; KF f; } ks[] = {{"16 add", k_a16}, {"16 pk_min", k_m16}, {"add/min alternating", k_am1},
      {"8 add then 8 min", k_am8}, {"runs of 4", k_am4}, {"runs of 2", k_am2}, {"dep add->min x8", k_dep1},
      {"dep 4 add, 4 min x2", k_dep4}, {"body mix interleaved", k_mixa}, {"body mix fast first", k_mixb},
      {"body mix slow first", k_mixc}};
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  uint32_t* out;
  hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double ghz = 2.4;
  for (int rep = 0; rep < 2; rep++)
  for (int wps : {2, 4}) {
    const int blocks = cus * wps;
    for (auto& k : ks) {
      k.f<<<blocks, 256>>>(out, 7);
      hipEventRecord(a);
      k.f<<<blocks, 256>>>(out, 7);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double ninst = (double)wps * ITERS * 16;      // per SIMD
      printf("wps=%d %-24s %7.3f ms  %6.2f cyc/inst/SIMD  %6.1f cyc per 16\n", wps, k.n, ms,
             ms * 1e-3 * ghz * 1e9 / ninst, ms * 1e-3 * ghz * 1e9 / ninst * 16); fflush(stdout);
    }
  }
  return 0;
}
