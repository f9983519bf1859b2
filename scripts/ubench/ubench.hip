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
             r12 = r0 + 12, r13 = r0 + 13, r14 = r0 + 14, r15 = r0 + 15, c = s * 3u + threadIdx.x; \
    for (int it = 0; it < ITERS; it++) {                                                   \
      asm volatile(R16(INS) : [r0] "+v"(r0), [r1] "+v"(r1), [r2] "+v"(r2), [r3] "+v"(r3),  \
                   [r4] "+v"(r4), [r5] "+v"(r5), [r6] "+v"(r6), [r7] "+v"(r7), [r8] "+v"(r8), \
                   [r9] "+v"(r9), [r10] "+v"(r10), [r11] "+v"(r11), [r12] "+v"(r12),       \
                   [r13] "+v"(r13), [r14] "+v"(r14), [r15] "+v"(r15)                        \
                   : [c] "v"(c), [s] "s"(s) : "vcc", "s0", "memory");                            \
    }                                                                                      \
    out[blockIdx.x * 256 + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7 ^ r8 ^ r9 ^ r10 ^ \
        r11 ^ r12 ^ r13 ^ r14 ^ r15;                                                       \
  }

#define I_ADD(i) "v_add_u32 %[r" #i "], %[r" #i "], %[c]\n\t"
#define I_PKADD(i) "v_pk_add_u16 %[r" #i "], %[r" #i "], %[c]\n\t"
#define I_PKMIN(i) "v_pk_min_u16 %[r" #i "], %[r" #i "], %[c]\n\t"
#define I_PKADDSW(i) "v_pk_add_u16 %[r" #i "], %[r" #i "], %[c] op_sel:[1,0] op_sel_hi:[0,1]\n\t"
#define I_XAD(i) "v_xad_u32 %[r" #i "], %[r" #i "], %[c], %[s]\n\t"
#define I_SAD(i) "v_sad_u32 %[r" #i "], 28, %[r" #i "], %[c]\n\t"
#define I_ANDOR(i) "v_and_or_b32 %[r" #i "], %[r" #i "], %[s], %[c]\n\t"
#define I_ALIGN(i) "v_alignbit_b32 %[r" #i "], %[c], %[r" #i "], 1\n\t"
#define I_ADDDPP(i) "v_add_u32_dpp %[r" #i "], %[c], %[r" #i "] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
#define I_MOVDPP8(i) "v_mov_b32_dpp %[r" #i "], %[c] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
#define I_MINDPP(i) "v_min_u32_dpp %[r" #i "], %[c], %[r" #i "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
#define I_CNDDPP(i) "v_cndmask_b32_dpp %[r" #i "], %[c], %[r" #i "], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
#define I_ADDC(i) "v_addc_co_u32 %[r" #i "], vcc, %[r" #i "], %[r" #i "], vcc\n\t"
#define I_CMP16(i) "v_cmp_eq_u16 vcc, %[r" #i "], %[c]\n\t"
#define I_CMP16SDWA(i) "v_cmp_eq_u16_sdwa vcc, %[r" #i "], %[c] src0_sel:WORD_1 src1_sel:WORD_1\n\t"
#define I_MUL24(i) "v_mul_u32_u24 %[r" #i "], %[r" #i "], %[c]\n\t"
#define I_BFI(i) "v_bfi_b32 %[r" #i "], %[c], %[r" #i "], %[s]\n\t"
#define I_PERM(i) "v_perm_b32 %[r" #i "], %[s], %[r" #i "], %[c]\n\t"
#define I_PL32(i) "v_permlane32_swap_b32 %[r" #i "], %[c]\n\t"
#define I_PL16(i) "v_permlane16_swap_b32 %[r" #i "], %[c]\n\t"
#define I_READLANE(i) "v_readlane_b32 s0, %[r" #i "], 5\n\t"
#define I_SWZ(i) "ds_swizzle_b32 %[r" #i "], %[r" #i "] offset:0x401F\n\t"
#define I_BPERM(i) "ds_bpermute_b32 %[r" #i "], %[c], %[r" #i "]\n\t"
#define I_CMPU32(i) "v_cmp_eq_u32 vcc, %[r" #i "], %[c]\n\t"

DEFK(k_add, I_ADD) DEFK(k_pkadd, I_PKADD) DEFK(k_pkmin, I_PKMIN) DEFK(k_pkaddsw, I_PKADDSW)
DEFK(k_xad, I_XAD) DEFK(k_sad, I_SAD) DEFK(k_andor, I_ANDOR) DEFK(k_align, I_ALIGN)
DEFK(k_adddpp, I_ADDDPP) DEFK(k_movdpp8, I_MOVDPP8) DEFK(k_mindpp, I_MINDPP) DEFK(k_cnddpp, I_CNDDPP)
DEFK(k_addc, I_ADDC) DEFK(k_cmp16, I_CMP16) DEFK(k_cmp16sdwa, I_CMP16SDWA) DEFK(k_mul24, I_MUL24)
DEFK(k_bfi, I_BFI) DEFK(k_perm, I_PERM) DEFK(k_pl32, I_PL32) DEFK(k_pl16, I_PL16)
DEFK(k_readlane, I_READLANE) DEFK(k_swz, I_SWZ) DEFK(k_bperm, I_BPERM) DEFK(k_cmpu32, I_CMPU32)

typedef void (*KF)(uint32_t*, uint32_t);
int main() {
  struct { const char* n; KF f; } ks[] = {
      {"v_add_u32", k_add}, {"v_pk_add_u16", k_pkadd}, {"v_pk_min_u16", k_pkmin},
      {"v_pk_add_u16 opsel-swap", k_pkaddsw}, {"v_xad_u32", k_xad}, {"v_sad_u32", k_sad},
      {"v_and_or_b32", k_andor}, {"v_alignbit_b32", k_align}, {"v_add_u32_dpp qp", k_adddpp},
      {"v_mov_b32_dpp ror8", k_movdpp8}, {"v_min_u32_dpp ror8", k_mindpp}, {"v_cndmask_b32_dpp", k_cnddpp},
      {"v_addc_co_u32", k_addc}, {"v_cmp_eq_u16", k_cmp16}, {"v_cmp_eq_u16_sdwa", k_cmp16sdwa},
      {"v_mul_u32_u24", k_mul24}, {"v_bfi_b32", k_bfi}, {"v_perm_b32", k_perm},
      {"v_permlane32_swap", k_pl32}, {"v_permlane16_swap", k_pl16}, {"v_readlane_b32", k_readlane},
      {"ds_swizzle_b32", k_swz}, {"ds_bpermute_b32", k_bperm},
      {"v_cmp_eq_u32", k_cmpu32}};
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
             ms * 1e-3 * ghz * 1e9 / inst_per_simd, ghz);
      fflush(stdout);
    }
  }
  return 0;
}
