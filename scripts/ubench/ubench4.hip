// gfx950 issue-cost microbenchmark, round 2: does a VOP2 instruction keep its cheap issue
// cost (~2.5 cycles per wave64, profiles/r01_ubench_isa_costs.log) inside a mixed stream?
// Sequences of the Viterbi column (tests/vit3_model.py step5) in different instruction
// orders, plus synthetic pairs.  Reports cycles per sequence instance per wave per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048

// ---- synthetic sequences: 8 independent registers a0..a7, c = VGPR operand, s = SGPR
#define SYN(NAME, BODY)                                                                     \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t s) {                  \
    uint32_t a0 = threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3, a4 = a0 + 4, a5 = a0 + 5, \
             a6 = a0 + 6, a7 = a0 + 7, c = s * 3u + threadIdx.x;                             \
    for (int it = 0; it < ITERS; it++) {                                                    \
      asm volatile(BODY BODY BODY BODY                                                      \
                   : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3), [a4] "+v"(a4), \
                     [a5] "+v"(a5), [a6] "+v"(a6), [a7] "+v"(a7), [c] "+v"(c)                \
                   : [s] "s"(s) : "vcc");                                                    \
    }                                                                                       \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;            \
  }

// 8 adds (4 pairs) + 8 pk_min, grouped by type
SYN(s_grouped,
    "v_add_u32 %[a0], %[c], %[a0]\n\tv_add_u32 %[a1], %[c], %[a1]\n\t"
    "v_add_u32 %[a2], %[c], %[a2]\n\tv_add_u32 %[a3], %[c], %[a3]\n\t"
    "v_pk_min_u16 %[a4], %[c], %[a4]\n\tv_pk_min_u16 %[a5], %[c], %[a5]\n\t"
    "v_pk_min_u16 %[a6], %[c], %[a6]\n\tv_pk_min_u16 %[a7], %[c], %[a7]\n\t")
// the same 8 alternating
SYN(s_alt,
    "v_add_u32 %[a0], %[c], %[a0]\n\tv_pk_min_u16 %[a4], %[c], %[a4]\n\t"
    "v_add_u32 %[a1], %[c], %[a1]\n\tv_pk_min_u16 %[a5], %[c], %[a5]\n\t"
    "v_add_u32 %[a2], %[c], %[a2]\n\tv_pk_min_u16 %[a6], %[c], %[a6]\n\t"
    "v_add_u32 %[a3], %[c], %[a3]\n\tv_pk_min_u16 %[a7], %[c], %[a7]\n\t")
// pairs of adds between pk_mins: add add min add add min ...
SYN(s_pairs,
    "v_add_u32 %[a0], %[c], %[a0]\n\tv_add_u32 %[a1], %[c], %[a1]\n\tv_pk_min_u16 %[a4], %[c], %[a4]\n\t"
    "v_pk_min_u16 %[a5], %[c], %[a5]\n\tv_add_u32 %[a2], %[c], %[a2]\n\tv_add_u32 %[a3], %[c], %[a3]\n\t"
    "v_pk_min_u16 %[a6], %[c], %[a6]\n\tv_pk_min_u16 %[a7], %[c], %[a7]\n\t")
// 8 adds, dependent in pairs (a0 += c; a0 += c)
SYN(s_dep_adds,
    "v_add_u32 %[a0], %[c], %[a0]\n\tv_add_u32 %[a0], %[c], %[a0]\n\t"
    "v_add_u32 %[a1], %[c], %[a1]\n\tv_add_u32 %[a1], %[c], %[a1]\n\t"
    "v_add_u32 %[a2], %[c], %[a2]\n\tv_add_u32 %[a2], %[c], %[a2]\n\t"
    "v_add_u32 %[a3], %[c], %[a3]\n\tv_add_u32 %[a3], %[c], %[a3]\n\t")
// 8 independent adds
SYN(s_adds,
    "v_add_u32 %[a0], %[c], %[a0]\n\tv_add_u32 %[a1], %[c], %[a1]\n\t"
    "v_add_u32 %[a2], %[c], %[a2]\n\tv_add_u32 %[a3], %[c], %[a3]\n\t"
    "v_add_u32 %[a4], %[c], %[a4]\n\tv_add_u32 %[a5], %[c], %[a5]\n\t"
    "v_add_u32 %[a6], %[c], %[a6]\n\tv_add_u32 %[a7], %[c], %[a7]\n\t")
// 8 independent pk_min
SYN(s_mins,
    "v_pk_min_u16 %[a0], %[c], %[a0]\n\tv_pk_min_u16 %[a1], %[c], %[a1]\n\t"
    "v_pk_min_u16 %[a2], %[c], %[a2]\n\tv_pk_min_u16 %[a3], %[c], %[a3]\n\t"
    "v_pk_min_u16 %[a4], %[c], %[a4]\n\tv_pk_min_u16 %[a5], %[c], %[a5]\n\t"
    "v_pk_min_u16 %[a6], %[c], %[a6]\n\tv_pk_min_u16 %[a7], %[c], %[a7]\n\t")
// 8 v_min_u16 (VOP2, low half only) + sdwa on the high half
SYN(s_min16_sdwa,
    "v_min_u16 %[a0], %[c], %[a0]\n\tv_min_u16_sdwa %[a0], %[c], %[a0] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n\t"
    "v_min_u16 %[a1], %[c], %[a1]\n\tv_min_u16_sdwa %[a1], %[c], %[a1] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n\t"
    "v_min_u16 %[a2], %[c], %[a2]\n\tv_min_u16_sdwa %[a2], %[c], %[a2] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n\t"
    "v_min_u16 %[a3], %[c], %[a3]\n\tv_min_u16_sdwa %[a3], %[c], %[a3] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n\t")
// 8 v_perm with VGPR operands / with an SGPR operand
SYN(s_perm_v,
    "v_perm_b32 %[a0], %[c], %[a0], %[c]\n\tv_perm_b32 %[a1], %[c], %[a1], %[c]\n\t"
    "v_perm_b32 %[a2], %[c], %[a2], %[c]\n\tv_perm_b32 %[a3], %[c], %[a3], %[c]\n\t"
    "v_perm_b32 %[a4], %[c], %[a4], %[c]\n\tv_perm_b32 %[a5], %[c], %[a5], %[c]\n\t"
    "v_perm_b32 %[a6], %[c], %[a6], %[c]\n\tv_perm_b32 %[a7], %[c], %[a7], %[c]\n\t")
SYN(s_perm_s,
    "v_perm_b32 %[a0], %[s], %[a0], %[c]\n\tv_perm_b32 %[a1], %[s], %[a1], %[c]\n\t"
    "v_perm_b32 %[a2], %[s], %[a2], %[c]\n\tv_perm_b32 %[a3], %[s], %[a3], %[c]\n\t"
    "v_perm_b32 %[a4], %[s], %[a4], %[c]\n\tv_perm_b32 %[a5], %[s], %[a5], %[c]\n\t"
    "v_perm_b32 %[a6], %[s], %[a6], %[c]\n\tv_perm_b32 %[a7], %[s], %[a7], %[c]\n\t")
// 8 v_sub_u32_dpp (row_ror:8) independent
SYN(s_subdpp,
    "v_sub_u32_dpp %[a0], %[c], %[a0] row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
    "v_sub_u32_dpp %[a1], %[c], %[a1] row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
    "v_sub_u32_dpp %[a2], %[c], %[a2] row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
    "v_sub_u32_dpp %[a3], %[c], %[a3] row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
    "v_sub_u32_dpp %[a4], %[c], %[a4] row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
    "v_sub_u32_dpp %[a5], %[c], %[a5] row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
    "v_sub_u32_dpp %[a6], %[c], %[a6] row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
    "v_sub_u32_dpp %[a7], %[c], %[a7] row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t")
// 8 and-with-literal in pairs
SYN(s_andlit,
    "v_and_b32 %[a0], 0xfffeffff, %[a0]\n\tv_and_b32 %[a1], 0xfffeffff, %[a1]\n\t"
    "v_and_b32 %[a2], 0xfffeffff, %[a2]\n\tv_and_b32 %[a3], 0xfffeffff, %[a3]\n\t"
    "v_and_b32 %[a4], 0xfffeffff, %[a4]\n\tv_and_b32 %[a5], 0xfffeffff, %[a5]\n\t"
    "v_and_b32 %[a6], 0xfffeffff, %[a6]\n\tv_and_b32 %[a7], 0xfffeffff, %[a7]\n\t")
// 8 v_mov_b32 (VOP1)
SYN(s_mov,
    "v_mov_b32 %[a0], %[c]\n\tv_mov_b32 %[a1], %[c]\n\tv_mov_b32 %[a2], %[c]\n\tv_mov_b32 %[a3], %[c]\n\t"
    "v_mov_b32 %[a4], %[c]\n\tv_mov_b32 %[a5], %[c]\n\tv_mov_b32 %[a6], %[c]\n\tv_mov_b32 %[a7], %[c]\n\t")
// 8 v_min_u32 VOP2 explicit _e32
SYN(s_minu32,
    "v_min_u32_e32 %[a0], %[c], %[a0]\n\tv_min_u32_e32 %[a1], %[c], %[a1]\n\t"
    "v_min_u32_e32 %[a2], %[c], %[a2]\n\tv_min_u32_e32 %[a3], %[c], %[a3]\n\t"
    "v_min_u32_e32 %[a4], %[c], %[a4]\n\tv_min_u32_e32 %[a5], %[c], %[a5]\n\t"
    "v_min_u32_e32 %[a6], %[c], %[a6]\n\tv_min_u32_e32 %[a7], %[c], %[a7]\n\t")
// 8 v_max_i16 / v_sub_u16 (VOP2 16-bit)
SYN(s_sub16,
    "v_sub_u16 %[a0], %[c], %[a0]\n\tv_sub_u16 %[a1], %[c], %[a1]\n\tv_sub_u16 %[a2], %[c], %[a2]\n\tv_sub_u16 %[a3], %[c], %[a3]\n\t"
    "v_sub_u16 %[a4], %[c], %[a4]\n\tv_sub_u16 %[a5], %[c], %[a5]\n\tv_sub_u16 %[a6], %[c], %[a6]\n\tv_sub_u16 %[a7], %[c], %[a7]\n\t")
// 8 v_lshrrev_b32 (VOP2 shift)
SYN(s_lshr,
    "v_lshrrev_b32 %[a0], %[c], %[a0]\n\tv_lshrrev_b32 %[a1], %[c], %[a1]\n\tv_lshrrev_b32 %[a2], %[c], %[a2]\n\tv_lshrrev_b32 %[a3], %[c], %[a3]\n\t"
    "v_lshrrev_b32 %[a4], %[c], %[a4]\n\tv_lshrrev_b32 %[a5], %[c], %[a5]\n\tv_lshrrev_b32 %[a6], %[c], %[a6]\n\tv_lshrrev_b32 %[a7], %[c], %[a7]\n\t")
// 8 v_max_u32 / v_min_i32
SYN(s_mini32,
    "v_min_i32 %[a0], %[c], %[a0]\n\tv_min_i32 %[a1], %[c], %[a1]\n\tv_min_i32 %[a2], %[c], %[a2]\n\tv_min_i32 %[a3], %[c], %[a3]\n\t"
    "v_min_i32 %[a4], %[c], %[a4]\n\tv_min_i32 %[a5], %[c], %[a5]\n\tv_min_i32 %[a6], %[c], %[a6]\n\tv_min_i32 %[a7], %[c], %[a7]\n\t")
// 8 v_add_u16 with DPP
SYN(s_add16dpp,
    "v_add_u16_dpp %[a0], %[c], %[a0] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
    "v_add_u16_dpp %[a1], %[c], %[a1] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
    "v_add_u16_dpp %[a2], %[c], %[a2] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
    "v_add_u16_dpp %[a3], %[c], %[a3] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
    "v_add_u16_dpp %[a4], %[c], %[a4] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
    "v_add_u16_dpp %[a5], %[c], %[a5] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
    "v_add_u16_dpp %[a6], %[c], %[a6] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
    "v_add_u16_dpp %[a7], %[c], %[a7] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t")

// ---- the Viterbi column (4 DPP phases per loop iteration), 2 dwords per lane
// M = a0/a1 (metrics), T = a2/a3, BX = a4/a5, X = a6/a7, Z = v240/v241; P = c; sel = v242/v243
#define COLA(CTRL, LIT)                                                                      \
  "v_perm_b32 %[a4], %[s], %[c], v242\n\t"                                                   \
  "v_perm_b32 %[a5], %[s], %[c], v243\n\t"                                                   \
  "v_add_u32 %[a6], %[a4], %[a2]\n\t"                                                        \
  "v_sub_u32_dpp v240, %[a2], %[a4] " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"   \
  "v_add_u32 %[a7], %[a5], %[a3]\n\t"                                                        \
  "v_add_u32 v240, " LIT ", v240\n\t"                                                        \
  "v_sub_u32_dpp v241, %[a3], %[a5] " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"   \
  "v_add_u32 v241, " LIT ", v241\n\t"                                                        \
  "v_pk_min_u16 %[a0], %[a6], v240\n\t"                                                      \
  "v_pk_min_u16 %[a1], %[a7], v241\n\t"                                                      \
  "v_and_b32 %[a2], 0xfffeffff, %[a0]\n\t"                                                   \
  "v_and_b32 %[a3], 0xfffeffff, %[a1]\n\t"
#define COLB(CTRL, LIT)                                                                      \
  "v_perm_b32 %[a4], %[s], %[c], v242\n\t"                                                   \
  "v_perm_b32 %[a5], %[s], %[c], v243\n\t"                                                   \
  "v_sub_u32_dpp v240, %[a2], %[a4] " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"   \
  "v_sub_u32_dpp v241, %[a3], %[a5] " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"   \
  "v_add_u32 %[a6], %[a4], %[a2]\n\t"                                                        \
  "v_add_u32 %[a7], %[a5], %[a3]\n\t"                                                        \
  "v_add_u32 v240, " LIT ", v240\n\t"                                                        \
  "v_add_u32 v241, " LIT ", v241\n\t"                                                        \
  "v_pk_min_u16 %[a0], %[a6], v240\n\t"                                                      \
  "v_pk_min_u16 %[a1], %[a7], v241\n\t"                                                      \
  "v_and_b32 %[a2], 0xfffeffff, %[a0]\n\t"                                                   \
  "v_and_b32 %[a3], 0xfffeffff, %[a1]\n\t"
// B with the perm constant in a VGPR (v244) instead of an SGPR
#define COLC(CTRL, LIT)                                                                      \
  "v_perm_b32 %[a4], v244, %[c], v242\n\t"                                                   \
  "v_perm_b32 %[a5], v244, %[c], v243\n\t"                                                   \
  "v_sub_u32_dpp v240, %[a2], %[a4] " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"   \
  "v_sub_u32_dpp v241, %[a3], %[a5] " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"   \
  "v_add_u32 %[a6], %[a4], %[a2]\n\t"                                                        \
  "v_add_u32 %[a7], %[a5], %[a3]\n\t"                                                        \
  "v_add_u32 v240, " LIT ", v240\n\t"                                                        \
  "v_add_u32 v241, " LIT ", v241\n\t"                                                        \
  "v_pk_min_u16 %[a0], %[a6], v240\n\t"                                                      \
  "v_pk_min_u16 %[a1], %[a7], v241\n\t"                                                      \
  "v_and_b32 %[a2], 0xfffeffff, %[a0]\n\t"                                                   \
  "v_and_b32 %[a3], 0xfffeffff, %[a1]\n\t"
#define FOURCOLS(COL)                                                                        \
  COL("row_ror:8", "0x1c081c08") COL("row_mirror", "0xe100e10")                             \
  COL("quad_perm:[2,3,0,1]", "0xe200e20") COL("quad_perm:[1,0,3,2]", "0x1c401c40")
#define COLK(NAME, COL)                                                                     \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t s) {                  \
    uint32_t a0 = threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3, a4 = a0 + 4, a5 = a0 + 5, \
             a6 = a0 + 6, a7 = a0 + 7, c = s * 3u + threadIdx.x;                             \
    asm volatile("v_mov_b32 v242, 0x0c0d0c0e\n\tv_mov_b32 v243, 0x0c0f0c0d\n\tv_mov_b32 v244, 0x08080808" ::: "v242", "v243", "v244"); \
    for (int it = 0; it < ITERS; it++) {                                                    \
      asm volatile(FOURCOLS(COL)                                                            \
                   : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3), [a4] "+v"(a4), \
                     [a5] "+v"(a5), [a6] "+v"(a6), [a7] "+v"(a7), [c] "+v"(c)                \
                   : [s] "s"(s) : "v240", "v241", "v242", "v243", "v244");                    \
    }                                                                                       \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;            \
  }

// ---- column5 as the kernel issues it: per dword and, perm (BX), sub (C - BX), add, add_dpp, pk_min
#define C5TWO(CTRL, LIT)                                                                     \
  "v_and_b32 %[a0], 0xfffeffff, %[a0]\n\t"                                                 \
  "v_and_b32 %[a1], 0xfffeffff, %[a1]\n\t"                                                 \
  "v_perm_b32 %[a4], %[s], %[c], v242\n\t"                                                 \
  "v_perm_b32 %[a5], %[s], %[c], v243\n\t"                                                 \
  "v_sub_u32 %[a6], " LIT ", %[a4]\n\t"                                                    \
  "v_sub_u32 %[a7], " LIT ", %[a5]\n\t"                                                    \
  "v_add_u32 %[a4], %[a0], %[a4]\n\t"                                                      \
  "v_add_u32 %[a5], %[a1], %[a5]\n\t"                                                      \
  "v_add_u32_dpp %[a6], %[a0], %[a6] " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t" \
  "v_add_u32_dpp %[a7], %[a1], %[a7] " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t" \
  "v_pk_min_u16 %[a0], %[a4], %[a6]\n\t"                                                   \
  "v_pk_min_u16 %[a1], %[a5], %[a7]\n\t"
#define C5ONE(CTRL, LIT)                                                                     \
  "v_and_b32 %[a0], 0xfffeffff, %[a0]\n\t"                                                 \
  "v_perm_b32 %[a4], %[s], %[c], v242\n\t"                                                 \
  "v_sub_u32 %[a6], " LIT ", %[a4]\n\t"                                                    \
  "v_add_u32 %[a4], %[a0], %[a4]\n\t"                                                      \
  "v_add_u32_dpp %[a6], %[a0], %[a6] " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t" \
  "v_pk_min_u16 %[a0], %[a4], %[a6]\n\t"
COLK(c5_two_dwords, C5TWO)
COLK(c5_one_dword, C5ONE)
COLK(c_compiler_order, COLA)
COLK(c_paired, COLB)
COLK(c_paired_vperm, COLC)

typedef void (*KF)(uint32_t*, uint32_t);
int main() {
  struct { const char* n; KF f; int per; } ks[] = {
      {"8: 4 add + 4 pk_min grouped", s_grouped, 8}, {"8: add/pk_min alternating", s_alt, 8},
      {"8: add add min min x2", s_pairs, 8}, {"8: adds dependent in pairs", s_dep_adds, 8},
      {"8: independent adds", s_adds, 8}, {"8: independent pk_min", s_mins, 8},
      {"8: v_min_u16 + sdwa hi", s_min16_sdwa, 8}, {"8: v_perm vgpr", s_perm_v, 8},
      {"8: v_perm sgpr", s_perm_s, 8}, {"8: v_sub_u32_dpp", s_subdpp, 8}, {"8: v_and literal", s_andlit, 8},
      {"8: v_mov_b32", s_mov, 8}, {"8: v_min_u32_e32", s_minu32, 8}, {"8: v_sub_u16", s_sub16, 8},
      {"8: v_lshrrev_b32 vgpr", s_lshr, 8}, {"8: v_min_i32", s_mini32, 8}, {"8: v_add_u16_dpp", s_add16dpp, 8},
      {"col x4: compiler order", c_compiler_order, 4}, {"col x4: paired VOP2", c_paired, 4},
      {"col x4: paired, perm const vgpr", c_paired_vperm, 4},
      {"col5 x4: two dwords (4 pkts/wave)", c5_two_dwords, 4}, {"col5 x4: one dword (2 pkts/wave)", c5_one_dword, 4}};
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  uint32_t* out;
  hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double ghz = 2.4;
  for (int wps : {1, 2, 3, 4, 8}) {
    const int blocks = cus * wps;
    for (auto& k : ks) {
      k.f<<<blocks, 256>>>(out, 7);
      hipEventRecord(a);
      k.f<<<blocks, 256>>>(out, 7);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double units = (double)wps * ITERS * 4;     // sequence instances per SIMD
      const double cyc = ms * 1e-3 * ghz * 1e9 / units;
      const int ninst = k.per == 8 ? 8 : (k.f == c5_one_dword ? 24 : 48);   // instructions per instance
      printf("wps=%d %-36s %7.3f ms %7.2f cyc/instance %5.2f cyc/inst\n", wps, k.n, ms, cyc, cyc / ninst);
      fflush(stdout);
    }
  }
  return 0;
}
