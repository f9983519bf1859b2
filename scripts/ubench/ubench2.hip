// Instruction-throughput microbenchmark for gfx950 (design input for the Viterbi kernel).
// Each kernel runs ITERS x 16 independent copies of one instruction per wave; the grid fills
// every SIMD with W waves.  Reports cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define ITERS 4096
#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

#define DEFK(NAME, INS)                                                                    \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t s) {                 \
    uint32_t r0 = threadIdx.x, r1 = r0 ^ 1, r2 = r0 ^ 2, r3 = r0 ^ 3, r4 = r0 + 4, r5 = r0 + 5, \
             r6 = r0 + 6, r7 = r0 + 7, r8 = r0 + 8, r9 = r0 + 9, r10 = r0 + 10, r11 = r0 + 11, \
             r12 = r0 + 12, r13 = r0 + 13, r14 = r0 + 14, r15 = r0 + 15, c = s * 3u + threadIdx.x; uint32_t t = s; \
    for (int it = 0; it < ITERS; it++) {                                                   \
      asm volatile(R16(INS) : [r0] "+v"(r0), [t] "+s"(t), [c] "+v"(c), [r1] "+v"(r1), [r2] "+v"(r2), [r3] "+v"(r3),  \
                   [r4] "+v"(r4), [r5] "+v"(r5), [r6] "+v"(r6), [r7] "+v"(r7), [r8] "+v"(r8), \
                   [r9] "+v"(r9), [r10] "+v"(r10), [r11] "+v"(r11), [r12] "+v"(r12),       \
                   [r13] "+v"(r13), [r14] "+v"(r14), [r15] "+v"(r15)                        \
                   : [s] "s"(s) : "vcc", "scc", "v250", "v251", "v252", "v253", "memory");                            \
    }                                                                                      \
    out[blockIdx.x * 256 + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7 ^ r8 ^ r9 ^ r10 ^ \
        r11 ^ r12 ^ r13 ^ r14 ^ r15;                                                       \
  }

#define J0(i) "v_xor_b32 %[r" #i "], %[c], %[r" #i "]\n\t"
DEFK(j0, J0)
#define J1(i) "v_and_b32 %[r" #i "], %[c], %[r" #i "]\n\t"
DEFK(j1, J1)
#define J2(i) "v_or_b32 %[r" #i "], %[c], %[r" #i "]\n\t"
DEFK(j2, J2)
#define J3(i) "v_min_u32 %[r" #i "], %[c], %[r" #i "]\n\t"
DEFK(j3, J3)
#define J4(i) "v_sub_u32 %[r" #i "], %[c], %[r" #i "]\n\t"
DEFK(j4, J4)
#define J5(i) "v_lshlrev_b32 %[r" #i "], 1, %[r" #i "]\n\t"
DEFK(j5, J5)
#define J6(i) "v_add_u32 %[r" #i "], %[s], %[r" #i "]\n\t"
DEFK(j6, J6)
#define J7(i) "v_add_u32 %[r" #i "], 0x1c001c, %[r" #i "]\n\t"
DEFK(j7, J7)
#define J8(i) "v_add_u16 %[r" #i "], %[c], %[r" #i "]\n\t"
DEFK(j8, J8)
#define J9(i) "v_min_u16 %[r" #i "], %[c], %[r" #i "]\n\t"
DEFK(j9, J9)
#define J10(i) "v_cndmask_b32 %[r" #i "], %[c], %[r" #i "], vcc\n\t"
DEFK(j10, J10)
#define J11(i) "v_cndmask_b32_dpp %[r" #i "], %[c], %[r" #i "], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_add_u32 %[c], 1, %[c]\n\t"
DEFK(j11, J11)
#define J12(i) "v_cndmask_b32_dpp %[r" #i "], %[c], %[r" #i "], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_xad_u32 v250, %[c], %[c], %[s]\n\tv_xad_u32 v251, %[c], %[c], %[s]\n\tv_xad_u32 v252, %[c], %[c], %[s]\n\tv_xad_u32 v253, %[c], %[c], %[s]\n\t"
DEFK(j12, J12)
#define J13(i) "v_xad_u32 v250, %[c], %[c], %[s]\n\tv_xad_u32 v251, %[c], %[c], %[s]\n\tv_xad_u32 v252, %[c], %[c], %[s]\n\tv_xad_u32 v253, %[c], %[c], %[s]\n\t"
DEFK(j13, J13)
#define J14(i) "v_min_u32_dpp %[r" #i "], %[c], %[r" #i "] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
DEFK(j14, J14)
#define J15(i) "v_min_u32_dpp %[r" #i "], %[c], %[r" #i "] row_ror:4 row_mask:0xf bank_mask:0xa\n\t"
DEFK(j15, J15)
#define J16(i) "v_add_u32 %[r" #i "], %[c], %[r" #i "]\n\tv_xad_u32 v250, %[c], %[c], %[s]\n\t"
DEFK(j16, J16)
#define J17(i) "v_add_u32 %[r" #i "], %[c], %[r" #i "]\n\tv_pk_add_u16 v250, %[c], %[c]\n\t"
DEFK(j17, J17)
#define J18(i) "v_pk_add_u16 %[r" #i "], %[s], %[r" #i "]\n\t"
DEFK(j18, J18)
#define J19(i) "v_pk_sub_u16 %[r" #i "], %[c], %[r" #i "]\n\t"
DEFK(j19, J19)
#define J20(i) "v_pk_max_u16 %[r" #i "], %[c], %[r" #i "]\n\t"
DEFK(j20, J20)
#define J21(i) "v_addc_co_u32 %[r" #i "], vcc, %[c], %[r" #i "], vcc\n\t"
DEFK(j21, J21)
#define J22(i) "v_add_f32 %[r" #i "], %[c], %[r" #i "]\n\t"
DEFK(j22, J22)
#define J23(i) "v_add_f32 %[r" #i "], %[s], %[r" #i "]\n\t"
DEFK(j23, J23)
#define J24(i) "v_add3_u32 %[r" #i "], %[c], %[r" #i "], %[s]\n\t"
DEFK(j24, J24)
#define J25(i) "v_lshl_or_b32 %[r" #i "], %[r" #i "], 1, %[c]\n\t"
DEFK(j25, J25)
#define J26(i) "v_add_u32 %[r" #i "], %[c], %[r" #i "]\n\ts_add_u32 %[t], %[t], %[s]\n\t"
DEFK(j26, J26)
#define J27(i) "v_mov_b32_dpp %[r" #i "], %[c] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
DEFK(j27, J27)
#define J28(i) "v_readfirstlane_b32 %[t], %[r" #i "]\n\t"
DEFK(j28, J28)
typedef void (*KF)(uint32_t*, uint32_t);
int main() {
  struct { const char* n; KF f; } ks[] = {{"v_xor_b32", j0}, {"v_and_b32", j1}, {"v_or_b32", j2}, {"v_min_u32", j3}, {"v_sub_u32", j4}, {"v_lshlrev_b32", j5}, {"v_add_u32 sgpr", j6}, {"v_add_u32 literal", j7}, {"v_add_u16", j8}, {"v_min_u16", j9}, {"v_cndmask_b32 vop2", j10}, {"v_cndmask_b32_dpp+v_add", j11}, {"v_cndmask_dpp+4 vop3", j12}, {"4 vop3 alone", j13}, {"v_min_u32_dpp qp", j14}, {"v_min_u32_dpp bankmask", j15}, {"v_add+v_xad alt", j16}, {"v_add+v_pk_add alt", j17}, {"v_pk_add_u16 sgpr", j18}, {"v_pk_sub_u16", j19}, {"v_pk_max_u16", j20}, {"v_addc_co_u32 vop2", j21}, {"v_add_f32", j22}, {"v_add_f32 sgpr", j23}, {"v_add3_u32", j24}, {"v_lshl_or_b32", j25}, {"s_add (SALU) + v_add", j26}, {"v_mov_b32_dpp qp", j27}, {"v_readfirstlane", j28}};
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  uint32_t* out;
  hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double ghz = 2.4;
  for (int wps : {2, 4, 8}) {          // waves per SIMD
    const int blocks = cus * wps;         // 256-thread block = 4 waves = one per SIMD
    for (auto& k : ks) {
      k.f<<<blocks, 256>>>(out, 7);
      hipEventRecord(a);
      k.f<<<blocks, 256>>>(out, 7);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double inst_per_simd = (double)wps * ITERS * 16;
      printf("wps=%d %-26s %7.3f ms  %6.2f cyc/wave-inst/SIMD (@%.1fGHz)\n", wps, k.n, ms,
             ms * 1e-3 * ghz * 1e9 / inst_per_simd, ghz); fflush(stdout);
    }
  }
  return 0;
}
