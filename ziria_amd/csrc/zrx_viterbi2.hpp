// Batched Viterbi brick, v2: the MI355X-native layout.
//
// Same results as the brick driver loop (csrc/sora_ext_viterbi.cpp:66-153 over
// csrc/viterbicore.hpp) bit for bit, organised for a 64-wide wave:
//
//  * one packet per wave; lane L is a storage POSITION, not a state.  After t trellis
//    columns, position L holds state rotl6^t(L) (6-bit rotate).  One column maps the pair
//    {j, j+32} to {2j, 2j+1} = {rotl6(j), rotl6(j+32)}, so every position keeps its own
//    metric and only needs the metric of its butterfly partner, which sits at lane
//    L ^ (1 << (5 - t mod 6)).  Partners at distance 1, 2, 8 are fetched inside the select
//    instruction with DPP (quad_perm / row_ror); distances 4 and 16 use ds_swizzle and 32
//    ds_bpermute (LDS crossbar, no LDS memory).
//  * add-compare-select on the reference's u8 metric with the survivor marker in bit 0
//    (viterbicore.hpp:105-147): X = m + bm_own, Y = m + (28|14 - bm_own) is this position's
//    candidate for its partner's new state; both are masked to (x & 0xFE) | marker with
//    marker = bit 5 of the own state (the branch index seen from the new state).
//    bm(v, e) = 2v XOR 14e reproduces VIT_MA / VIT_MB (viterbilut.h).
//  * survivors by register exchange: H (32 bits per position) holds the last 32 decisions
//    along the survivor path of the position's state (newest in bit 31).  H is snapshotted
//    to LDS at every column C = 6 (mod 32); decision d_c is the decoded bit c-7, so one
//    snapshot word along the path IS 4 output bytes.  The reference traceback
//    (viterbicore.hpp:170-239: signed-int16 argmin start, `lookahead` skipped columns,
//    bytes filled from the end) therefore becomes: argmin -> state at column T-look ->
//    8 dependent LDS reads per 256-bit window (state 32 columns back = bitreverse of the
//    low 6 bits of the word).
#pragma once
#include <utility>

#include "zrx_device.hpp"

namespace zrx {
namespace v2 {

constexpr int kSnapSlots = 16;                 // 16 x 32 columns of history (>= 288 needed)

__host__ __device__ constexpr uint32_t rotl6(uint32_t x, int k) {
  return k == 0 ? (x & 63u) : (((x << k) | (x >> (6 - k))) & 63u);
}
__host__ __device__ constexpr uint32_t rotr6(uint32_t x, int k) { return rotl6(x, (6 - k) % 6); }

// Per-position constants for phase ph (= column index mod 6 before the step).
struct Consts {
  uint32_t mA[6], mB[6], bm[6];
};
__device__ __forceinline__ Consts make_consts(int lane) {
  Consts C;
#pragma unroll
  for (int ph = 0; ph < 6; ph++) {
    const uint32_t j = rotl6((uint32_t)lane, ph);
    const uint32_t f = ((j >> 1) ^ (j >> 2) ^ (j >> 4)) & 1u;   // expected A of j -> rotl6(j)
    const uint32_t g = (j ^ (j >> 1) ^ (j >> 2)) & 1u;          // expected B
    C.mA[ph] = 14u * f;
    C.mB[ph] = 14u * g;
    C.bm[ph] = (j >> 5) & 1u;
  }
  return C;
}

// ---------------------------------------------------------------- one trellis column
#define ZRX_P1_FULL                                     \
  "v_xor_b32 %[t], %[b2], %[mB]\n\t"                    \
  "v_xad_u32 %[beta], %[a2], %[mA], %[t]\n\t"           \
  "v_sad_u32 %[Y], 28, %[beta], %[m]\n\t"               \
  "v_and_or_b32 %[Ym], %[Y], %[fe], %[bm]\n\t"          \
  "v_add_u32 %[X], %[m], %[beta]\n\t"                   \
  "v_and_or_b32 %[Xm], %[X], %[fe], %[bm]\n\t"
#define ZRX_P1_SINGLE                                   \
  "v_xor_b32 %[beta], %[a2], %[mA]\n\t"                 \
  "v_sad_u32 %[Y], 14, %[beta], %[m]\n\t"               \
  "v_and_or_b32 %[Ym], %[Y], %[fe], %[bm]\n\t"          \
  "v_add_u32 %[X], %[m], %[beta]\n\t"                   \
  "v_and_or_b32 %[Xm], %[X], %[fe], %[bm]\n\t"
// select with the partner fetched by DPP inside v_min / v_cndmask; Ym is written three
// instructions before its first DPP read (gfx9 needs two wait states).
#define ZRX_SEL_DPP(CTRL)                                                              \
  "v_min_u32_dpp %[m], %[Ym], %[Xm] " CTRL " row_mask:0xf bank_mask:0xf\n\t"           \
  "v_cmp_eq_u32 vcc, %[m], %[Xm]\n\t"                                                  \
  "v_cndmask_b32_dpp %[Hs], %[H], %[H], vcc " CTRL " row_mask:0xf bank_mask:0xf\n\t"   \
  "v_alignbit_b32 %[H], %[m], %[Hs], 1\n\t"

#define ZRX_OUTS [t] "=&v"(t), [beta] "=&v"(beta), [Y] "=&v"(Y), [Ym] "=&v"(Ym), [X] "=&v"(X), \
                 [Xm] "=&v"(Xm), [Hs] "=&v"(Hs), [m] "+v"(m), [H] "+v"(H)

// KIND 0: (a, b) on A and B; 1: a on A only; 2: a on B only.  a2 = 2a, b2 = 2b.
template <int PH, int KIND>
__device__ __forceinline__ void step(uint32_t& m, uint32_t& H, uint32_t a2, uint32_t b2, const Consts& C,
                                     uint32_t fe, uint32_t xaddr) {
  uint32_t t, beta, Y, Ym, X, Xm, Hs;
  const uint32_t mA = KIND == 2 ? C.mB[PH] : C.mA[PH];
  const uint32_t mB = C.mB[PH], bm = C.bm[PH];
  constexpr int K = 32 >> PH;                   // partner distance
  if constexpr (K == 1 || K == 2 || K == 8) {
#define ZRX_DO(P1, CTRL)                                                                   \
  asm volatile(P1 ZRX_SEL_DPP(CTRL)                                                       \
               : ZRX_OUTS                                                                  \
               : [a2] "s"(a2), [b2] "s"(b2), [mA] "v"(mA), [mB] "v"(mB), [bm] "v"(bm),     \
                 [fe] "s"(fe)                                                              \
               : "vcc")
    if constexpr (KIND == 0) {
      if constexpr (K == 1) ZRX_DO(ZRX_P1_FULL, "quad_perm:[1,0,3,2]");
      else if constexpr (K == 2) ZRX_DO(ZRX_P1_FULL, "quad_perm:[2,3,0,1]");
      else ZRX_DO(ZRX_P1_FULL, "row_ror:8");
    } else {
      if constexpr (K == 1) ZRX_DO(ZRX_P1_SINGLE, "quad_perm:[1,0,3,2]");
      else if constexpr (K == 2) ZRX_DO(ZRX_P1_SINGLE, "quad_perm:[2,3,0,1]");
      else ZRX_DO(ZRX_P1_SINGLE, "row_ror:8");
    }
#undef ZRX_DO
  } else if constexpr (K == 4) {
    // partner at lane ^ 4: banks 0,2 of each row read lane+4 (row_ror:12), banks 1,3 lane-4
    // (row_ror:4); two bank-masked DPP writes assemble the min and the H select.
#define ZRX_SEL4                                                                                    \
  "v_min_u32_dpp %[m], %[Ym], %[Xm] row_ror:12 row_mask:0xf bank_mask:0x5\n\t"                      \
  "v_min_u32_dpp %[m], %[Ym], %[Xm] row_ror:4 row_mask:0xf bank_mask:0xa\n\t"                       \
  "v_cmp_eq_u32 vcc, %[m], %[Xm]\n\t"                                                               \
  "v_cndmask_b32_dpp %[Hs], %[H], %[H], vcc row_ror:12 row_mask:0xf bank_mask:0x5\n\t"              \
  "v_cndmask_b32_dpp %[Hs], %[H], %[H], vcc row_ror:4 row_mask:0xf bank_mask:0xa\n\t"               \
  "v_alignbit_b32 %[H], %[m], %[Hs], 1\n\t"
    if constexpr (KIND == 0)
      asm volatile(ZRX_P1_FULL ZRX_SEL4 : ZRX_OUTS
                   : [a2] "s"(a2), [b2] "s"(b2), [mA] "v"(mA), [mB] "v"(mB), [bm] "v"(bm), [fe] "s"(fe) : "vcc");
    else
      asm volatile(ZRX_P1_SINGLE ZRX_SEL4 : ZRX_OUTS
                   : [a2] "s"(a2), [b2] "s"(b2), [mA] "v"(mA), [mB] "v"(mB), [bm] "v"(bm), [fe] "s"(fe) : "vcc");
#undef ZRX_SEL4
  } else {
    // partner at lane ^ 16 / ^ 32: v_permlane{16,32}_swap on copies leaves the partner's
    // value in the even/lower (second operand) or odd/upper (first operand) rows; row-masked
    // identity DPP writes pick per row.
    uint32_t YB, HA, HB;
#define ZRX_SELX(SWAP, RLO, RHI)                                                                    \
  "v_mov_b32 %[YB], %[Ym]\n\t"                                                                      \
  "v_mov_b32 %[HA], %[H]\n\t"                                                                       \
  "v_mov_b32 %[HB], %[H]\n\t"                                                                       \
  "s_nop 1\n\t"                                                                                     \
  SWAP " %[Ym], %[YB]\n\t"                                                                          \
  SWAP " %[HA], %[HB]\n\t"                                                                          \
  "s_nop 1\n\t"                                                                                     \
  "v_min_u32_dpp %[m], %[YB], %[Xm] quad_perm:[0,1,2,3] row_mask:" RLO " bank_mask:0xf\n\t"         \
  "v_min_u32_dpp %[m], %[Ym], %[Xm] quad_perm:[0,1,2,3] row_mask:" RHI " bank_mask:0xf\n\t"         \
  "v_cmp_eq_u32 vcc, %[m], %[Xm]\n\t"                                                               \
  "v_cndmask_b32_dpp %[Hs], %[HB], %[H], vcc quad_perm:[0,1,2,3] row_mask:" RLO " bank_mask:0xf\n\t" \
  "v_cndmask_b32_dpp %[Hs], %[HA], %[H], vcc quad_perm:[0,1,2,3] row_mask:" RHI " bank_mask:0xf\n\t" \
  "v_alignbit_b32 %[H], %[m], %[Hs], 1\n\t"
#define ZRX_OUTSX ZRX_OUTS, [YB] "=&v"(YB), [HA] "=&v"(HA), [HB] "=&v"(HB)
    if constexpr (K == 16) {
      if constexpr (KIND == 0)
        asm volatile(ZRX_P1_FULL ZRX_SELX("v_permlane16_swap_b32", "0x5", "0xa") : ZRX_OUTSX
                     : [a2] "s"(a2), [b2] "s"(b2), [mA] "v"(mA), [mB] "v"(mB), [bm] "v"(bm), [fe] "s"(fe) : "vcc");
      else
        asm volatile(ZRX_P1_SINGLE ZRX_SELX("v_permlane16_swap_b32", "0x5", "0xa") : ZRX_OUTSX
                     : [a2] "s"(a2), [b2] "s"(b2), [mA] "v"(mA), [mB] "v"(mB), [bm] "v"(bm), [fe] "s"(fe) : "vcc");
    } else {
      if constexpr (KIND == 0)
        asm volatile(ZRX_P1_FULL ZRX_SELX("v_permlane32_swap_b32", "0x3", "0xc") : ZRX_OUTSX
                     : [a2] "s"(a2), [b2] "s"(b2), [mA] "v"(mA), [mB] "v"(mB), [bm] "v"(bm), [fe] "s"(fe) : "vcc");
      else
        asm volatile(ZRX_P1_SINGLE ZRX_SELX("v_permlane32_swap_b32", "0x3", "0xc") : ZRX_OUTSX
                     : [a2] "s"(a2), [b2] "s"(b2), [mA] "v"(mA), [mB] "v"(mB), [bm] "v"(bm), [fe] "s"(fe) : "vcc");
    }
#undef ZRX_SELX
#undef ZRX_OUTSX
    (void)xaddr;
  }
}

// ---------------------------------------------------------------- wave helpers
__device__ __forceinline__ uint32_t wave_min_dpp(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));   // xor 1
  v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));   // xor 2
  v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, true));  // row_ror 4
  v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, true));  // row_ror 8
  const uint32_t r0 = __builtin_amdgcn_readlane((int)v, 0), r1 = __builtin_amdgcn_readlane((int)v, 16);
  const uint32_t r2 = __builtin_amdgcn_readlane((int)v, 32), r3 = __builtin_amdgcn_readlane((int)v, 48);
  return min(min(r0, r1), min(r2, r3));
}

// ---------------------------------------------------------------- traceback
// Output (in lane w) of word w of the window; nwords words, the last one holding `tailbits`
// (8..32) bits.  T: current column, look: skipped columns, cnt: output bits (multiple of 8).
struct TbOut { uint32_t word; int nbytes; };
__device__ __forceinline__ TbOut traceback(uint32_t m, uint32_t H, uint32_t T, uint32_t look, uint32_t cnt,
                                           int lane, const uint32_t* snap) {
  const int phT = (int)(T % 6u);
  const uint32_t s_lane = rotl6((uint32_t)lane, phT);
  int key = (int)(int16_t)(uint16_t)((m << 8) | (s_lane << 2));
  key = wave_min_i32(key);
  const uint32_t sstar = ((uint32_t)key >> 2) & 63u;
  const uint32_t Hs = (uint32_t)__builtin_amdgcn_readlane((int)H, (int)rotr6(sstar, phT));
  uint64_t XS = (uint64_t)sstar | ((uint64_t)__builtin_bitreverse32(Hs) << 6);
  const uint32_t Clast = T - look;                    // last output column
  const uint32_t r = (Clast - 6u) & 31u;              // bits past the last snapshot column
  const int nfull = (int)((cnt - r) >> 5);
  const int nwords = nfull + (r ? 1 : 0);
  uint32_t mine = 0;
  if (r) {                                            // columns (Clast-r, Clast] straight from H_T
    const uint32_t part = (Hs >> (32u - look - r)) & ((1u << r) - 1u);
    if (lane == nwords - 1) mine = part;
  }
  uint32_t C = Clast - r;                             // a snapshot column (C = 6 mod 32)
  uint32_t sC = (uint32_t)(XS >> (look + r)) & 63u;
  for (int w = nfull - 1; w >= 0; w--) {
    const uint32_t slot = (C >> 5) & (kSnapSlots - 1);
    const uint32_t W = snap[slot * 64 + rotr6(sC, (int)(C % 6u))];
    if (lane == w) mine = W;
    XS = (uint64_t)sC | ((uint64_t)__builtin_bitreverse32(W) << 6);
    sC = (uint32_t)(XS >> 32) & 63u;
    C -= 32;
  }
  TbOut o;
  o.word = mine;
  o.nbytes = lane < nfull ? 4 : (lane == nwords - 1 && r ? (int)(r >> 3) : 0);
  return o;
}

// ---------------------------------------------------------------- packet driver
// A body is 96 columns (lcm of the 6 label phases and the 32-column snapshot period), so
// phases, snapshot columns (6 mod 32) and normalize points (tr = 0 mod 8, checked after
// each group) sit at fixed positions in straight-line code; one body consumes one chunk of
// soft values (one dword per lane, broadcast by readlane).
struct Run {
  uint32_t tr, ob, tr_end, total_bytes, next;
  bool done;
};

template <int CR> struct Rate;
template <> struct Rate<0> { static constexpr int G = 2, steps = 1, groups = 96, chunk_dw = 48; };   // 1/2
template <> struct Rate<1> { static constexpr int G = 3, steps = 2, groups = 48, chunk_dw = 36; };   // 2/3
template <> struct Rate<2> { static constexpr int G = 4, steps = 3, groups = 32, chunk_dw = 32; };   // 3/4

// A partial traceback due inside a body is recorded here (slow path only) and run when the
// body ends; the final traceback ends the packet, so it runs on the live m and H.
struct Pending { uint32_t m, H, T, look; bool due; };

__device__ __forceinline__ void write_window(const TbOut& o, uint32_t first_byte, int lane, uint8_t* __restrict__ out) {
  uint8_t* d = out + first_byte + 4 * lane;
  for (int b = 0; b < o.nbytes; b++) d[b] = (uint8_t)(o.word >> (8 * b));
}

template <int CR>
struct Body {
  using RT = Rate<CR>;
  const Consts& C;
  uint32_t fe, xaddr;
  int lane;
  uint32_t* snap;
  __device__ __forceinline__ uint32_t soft2(uint32_t chunk, int idx) const {   // 2 x soft value idx
    const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)chunk, idx >> 2);
    return ((w >> (8 * (idx & 3))) & 0xFFu) << 1;
  }
  template <int COL, int KIND>
  __device__ __forceinline__ void col(uint32_t& m, uint32_t& H, uint32_t a2, uint32_t b2, uint32_t tr0) const {
    step<COL % 6, KIND>(m, H, a2, b2, C, fe, xaddr);
    if constexpr ((COL + 1) % 32 == 6)                 // snapshot column (tr0 = 0 mod 96)
      snap[(((tr0 + COL + 1) >> 5) & (kSnapSlots - 1)) * 64 + lane] = H;
  }
  template <int GI>
  __device__ __forceinline__ void group(uint32_t& m, uint32_t& H, uint32_t chunk, uint32_t tr0, int cn, Run& R,
                                        Pending& pend) const {
    constexpr int c0 = GI * RT::steps, s0 = GI * RT::G;
    // input exhausted (last chunk) or final traceback taken: the brick outputs nothing more
    if (__builtin_expect(s0 >= cn || R.done, 0)) return;
    if constexpr (CR == 0) {
      col<c0, 0>(m, H, soft2(chunk, s0), soft2(chunk, s0 + 1), tr0);
    } else if constexpr (CR == 1) {
      col<c0, 0>(m, H, soft2(chunk, s0), soft2(chunk, s0 + 1), tr0);
      col<c0 + 1, 1>(m, H, soft2(chunk, s0 + 2), 0, tr0);
    } else {
      col<c0, 0>(m, H, soft2(chunk, s0), soft2(chunk, s0 + 1), tr0);
      col<c0 + 1, 1>(m, H, soft2(chunk, s0 + 2), 0, tr0);
      col<c0 + 2, 2>(m, H, soft2(chunk, s0 + 3), 0, tr0);
    }
    constexpr int cend = c0 + RT::steps;               // columns done in this body
    if constexpr (cend % 8 == 0) m -= wave_min_dpp(m) & 0xFEu;   // sora_ext_viterbi.cpp:112-116
    // traceback schedule (:118-149); fast path = one compare against R.next
    const uint32_t tr = tr0 + cend;
    if (__builtin_expect(tr >= R.next, 0)) {
      if (tr >= R.tr_end) {
        R.done = true;
        R.tr = tr;
      } else {
        pend.m = m; pend.H = H; pend.T = tr; pend.look = 24u + ((tr - (R.ob + 286u)) & 7u); pend.due = true;
        R.ob += 256u;
        R.next = min(R.ob + 286u, R.tr_end);
      }
    }
  }
  template <int... GI>
  __device__ __forceinline__ void all(uint32_t& m, uint32_t& H, uint32_t chunk, uint32_t tr0, int cn, Run& R,
                                      Pending& pend, std::integer_sequence<int, GI...>) const {
    (group<GI>(m, H, chunk, tr0, cn, R, pend), ...);
  }
};

template <int CR>
__device__ __forceinline__ void run_packet(const uint8_t* __restrict__ sp, int n, Run& R, int lane,
                                           uint32_t* snap, uint8_t* __restrict__ out) {
  using RT = Rate<CR>;
  const Consts C = make_consts(lane);
  const Body<CR> B{C, (uint32_t)__builtin_amdgcn_readfirstlane(0xFE), (uint32_t)(lane ^ 32) << 2, lane, snap};
  uint32_t m = lane == 0 ? 0u : 48u;                  // ALL_INIT0 / ALL_INIT
  uint32_t H = 0;
  Pending pend;
  pend.due = false;
  pend.m = pend.H = pend.T = pend.look = 0;
  constexpr int CHUNK = RT::chunk_dw * 4;             // soft values per 96-column body
  const uint32_t* sp32 = (const uint32_t*)sp;
  uint32_t nxt = (lane < RT::chunk_dw && 4 * lane < n) ? sp32[lane] : 0u;
  uint32_t tr0 = 0;
  for (int base = 0; base < n && !R.done; base += CHUNK, tr0 += 96) {
    const uint32_t chunk = nxt;
    const int nb = base + CHUNK;
    nxt = (lane < RT::chunk_dw && nb + 4 * lane < n) ? sp32[nb / 4 + lane] : 0u;
    const int cn = min(CHUNK, n - base);
    B.all(m, H, chunk, tr0, cn, R, pend, std::make_integer_sequence<int, RT::groups>{});
    if (pend.due) {
      write_window(traceback(pend.m, pend.H, pend.T, pend.look, 256u, lane, snap), R.total_bytes, lane, out);
      R.total_bytes += 32u;
      pend.due = false;
    }
  }
  if (R.done) {                                       // final traceback at column R.tr
    const uint32_t cnt = R.tr_end - R.ob - 6u;
    if (cnt) write_window(traceback(m, H, R.tr, R.tr - R.tr_end, cnt, lane, snap), R.total_bytes, lane, out);
    R.total_bytes += cnt >> 3;
  }
}

}  // namespace v2

// vparams[4p..] = {frame_len, code_rate, soft_len, *}; out_bits[p] = bits written.
// Requires depth 256 (the only depth the WiFi RX uses: Viterbi.blk:34).
__global__ __launch_bounds__(256) void k_viterbi2(const uint8_t* __restrict__ soft, const int64_t* __restrict__ soft_off,
                                                  const int32_t* __restrict__ vparams, int npkts,
                                                  uint8_t* __restrict__ out, const int64_t* __restrict__ out_off,
                                                  int32_t* __restrict__ out_bits) {
  __shared__ uint32_t snap_all[4][v2::kSnapSlots * 64];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int p = blockIdx.x * 4 + wv;
  if (p >= npkts) return;
  const int32_t* vp = vparams + 4 * (int64_t)p;
  const int fl = __builtin_amdgcn_readfirstlane(vp[0]);
  const int cr = __builtin_amdgcn_readfirstlane(vp[1]);
  const int n = __builtin_amdgcn_readfirstlane(vp[2]);
  v2::Run R;
  R.tr = 0; R.ob = 0; R.tr_end = (uint32_t)fl * 8u + 6u; R.total_bytes = 0; R.done = false;
  R.next = min(286u, R.tr_end);
  const int64_t so = soft_off[p], oo = out_off[p];
  const uint8_t* sp = soft + __builtin_amdgcn_readfirstlane((int)(so & 0xFFFFFFFF)) +
                      ((int64_t)__builtin_amdgcn_readfirstlane((int)(so >> 32)) << 32);
  uint8_t* op = out + __builtin_amdgcn_readfirstlane((int)(oo & 0xFFFFFFFF)) +
                ((int64_t)__builtin_amdgcn_readfirstlane((int)(oo >> 32)) << 32);
  uint32_t* snap = snap_all[wv];
  if (n > 0) {
    if (cr == 0) v2::run_packet<0>(sp, n, R, lane, snap, op);
    else if (cr == 1) v2::run_packet<1>(sp, n, R, lane, snap, op);
    else if (cr == 2) v2::run_packet<2>(sp, n, R, lane, snap, op);
  }
  if (lane == 0) out_bits[p] = (int32_t)(R.total_bytes * 8u);
}

}  // namespace zrx
