// Batched Viterbi brick, v3: several packets per wave, the 64 trellis positions of a packet
// packed as kLanes lanes x kDw dwords x 2 16-bit halves (one "row" of kLanes lanes).
//
// Same results as the brick driver loop (csrc/sora_ext_viterbi.cpp:66-153 over
// csrc/viterbicore.hpp:105-239) bit for bit; tests/vit3_model.py (16-lane rows) and
// tests/vit8_model.py (8-lane rows, the default) restate the layout in numpy and are checked
// against the reference frames and the oracle on the CPU.
//
//  * Labels rotate, positions stay: after t columns position p holds state rotl6(p, t mod 6),
//    so one column maps every position's state j to rotl6(j) in place and the butterfly
//    partner (state j ^ 32) sits at position p ^ (1 << (5 - t mod 6)).  Position bit 0 is the
//    half, the next log2(kDw) bits the dword inside the lane (partners in registers), the
//    rest lane bits: 8-lane rows map position bits 3, 4, 5 to lane xor 1, 2, 7 (DPP
//    quad_perm, quad_perm, row_half_mirror), 16-lane rows bits 2..5 to lane xor 1, 2, 15, 8
//    (quad_perm, quad_perm, row_mirror, row_ror:8), so each cross-lane partner is ONE DPP
//    move inside the row.
//  * Half = [0][H >> 1][pad]: H = the reference's u8 metric with its marker bit cleared
//    (always even) in bits 14..8, the pad (bits 7..0) holds the decisions of the current
//    8-column cycle (column5).  The candidates of one column always differ in the marker,
//    so v_pk_min_u16 reproduces min_epu8 on (metric | marker) exactly and drags the path
//    history along with the winner (register exchange at no extra cost).  Every 8 columns the pads are stored to an
//    LDS ring indexed by state: one byte there = 8 decoded bits, so the reference traceback
//    (argmin of the signed (m<<8)|4s key, `lookahead` skipped columns, bytes from the end)
//    becomes an argmin plus one dependent LDS read per output byte.
//  * Branch metrics (halved, like H): P = [BM(A=0,B=0), BM(0,1), BM(1,0), BM(1,1)] / 2
//    (implicit depuncturing: A-only / B-only columns have their own P, :93-110) is built
//    once per 24-column body by the row's lanes and broadcast with ds_swizzle; a dword gets
//    its branch metrics with one v_perm (per-lane selector) — or shares another dword's when
//    the state bits its dword bits flip at this phase change no expected bit (bx_src) — and
//    its complement with one v_sub from a literal.
//  * Why 8-lane rows: the cost per row of everything outside the column (P broadcast, walk,
//    argmin, events) halves, one more partner phase is an in-register dword swap instead of
//    a DPP add, and more dwords share branch-metric words (14 v_perm per 6 columns for 8
//    states a lane instead of 10 for 4).  The LDS ring holds 16 rows per SIMD either way.
#pragma once
#include <utility>

#include "zrx_device.hpp"

namespace zrx {
namespace v3 {

#ifndef ZRX_VLANES
#define ZRX_VLANES 8
#endif
constexpr int kLanes = ZRX_VLANES;                     // lanes per row (packet): 8 or 16
static_assert(kLanes == 4 || kLanes == 8 || kLanes == 16, "rows are 4, 8 or 16 lanes");
constexpr int kDw = 32 / kLanes;                       // dwords per lane: 4 or 2
constexpr int kDwBits = kLanes == 4 ? 3 : kLanes == 8 ? 2 : 1;   // position bits 1..kDwBits = the dword
constexpr int kLaneBits = kLanes == 4 ? 2 : kLanes == 8 ? 3 : 4;
constexpr int kRowsWave = 64 / kLanes;                 // rows per wave
constexpr uint32_t kRowMask = (1u << kLanes) - 1u;     // a row's lanes in a ballot (shifted)
constexpr int kRing = 39;                 // snapshot slots of 8 columns per packet (>= 38)
constexpr int kRows = 4 * kRowsWave;      // packets per 256-thread block
constexpr int kSlotBytes = kRows * 64;
constexpr int kWavesPerSimd = kLanes == 4 ? 1 : kLanes == 8 ? 2 : 4;   // LDS ring: 16 rows per SIMD
constexpr uint32_t kNever = 0x7FFFFFFFu;

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 h2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t w32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }

__host__ __device__ constexpr uint32_t rotl6(uint32_t x, uint32_t k) {
  return k == 0 ? (x & 63u) : (((x << k) | (x >> (6u - k))) & 63u);
}
// 6-bit reversal: the snapshot ring is indexed by rev6(state), so the walk's next index is
// the low 6 bits of the byte it just read (next state = rev6(byte & 63)).
__host__ __device__ constexpr uint32_t rev6(uint32_t x) {
  return ((x & 1u) << 5) | ((x & 2u) << 3) | ((x & 4u) << 1) | ((x & 8u) >> 1) | ((x & 16u) >> 3) | ((x & 32u) >> 5);
}
// position held by (lane-in-row l, dword d, half h)
//   8 lanes:  lane = b3*1 ^ b4*2 ^ b5*7        16 lanes: lane = b2*1 ^ b3*2 ^ b4*15 ^ b5*8
__host__ __device__ constexpr uint32_t pos_of(uint32_t l, uint32_t d, uint32_t h) {
  if (kLanes == 4) return h | (d << 1) | ((l & 1u) << 4) | (((l >> 1) & 1u) << 5);   // lane = b4*1 ^ b5*2
  if (kLanes == 8) {
    const uint32_t b5 = (l >> 2) & 1u;
    const uint32_t b3 = (l & 1u) ^ b5, b4 = ((l >> 1) & 1u) ^ b5;
    return h | (d << 1) | (b3 << 3) | (b4 << 4) | (b5 << 5);
  }
  const uint32_t b4 = (l >> 2) & 1u;
  const uint32_t b2 = (l & 1u) ^ b4, b3 = ((l >> 1) & 1u) ^ b4, b5 = ((l >> 3) & 1u) ^ b4;
  return h | (d << 1) | (b2 << 2) | (b3 << 3) | (b4 << 4) | (b5 << 5);
}
// DPP control of the cross-lane partner for position bit pb (> kDwBits)
__host__ __device__ constexpr int partner_dpp(int pb) {
  return kLanes == 4 ? (pb == 5 ? 0x4E : 0xB1)
       : kLanes == 8 ? (pb == 5 ? 0x141 : pb == 4 ? 0x4E : 0xB1)
                     : (pb == 5 ? 0x128 : pb == 4 ? 0x140 : pb == 3 ? 0x4E : 0xB1);
}
#ifndef ZRX_BX_COMP
#define ZRX_BX_COMP 1
#endif
// Branch-metric word sharing (tests/vit8_model.py bx_source): the state bits dword d's
// position bits flip at phase ph; flipping state bit 3 changes neither expected bit, bit 5
// only the marker, bits 1 and 2 both A and B, bit 0 B, bit 4 A (encoding.blk:92-109).
// Returns -1 (own v_perm) or e | mk << 8: dword e's word, marker bits flipped when mk.
__host__ __device__ constexpr uint32_t dw_flips(int ph, int d) {
  uint32_t f = 0;
  for (int b = 0; b < kDwBits; b++)
    if ((d >> b) & 1) f ^= 1u << ((b + 1 + ph) % 6);
  return f;
}
__host__ __device__ constexpr int ab_flips(uint32_t f) {
  int a = 0, b = 0;
  for (int i = 0; i < 6; i++)
    if ((f >> i) & 1) { a ^= (i == 1 || i == 2 || i == 4); b ^= (i <= 2); }
  return 2 * a + b;
}
// Failing that, e | mk << 8 | 1 << 9 when dword e's states have both expected bits flipped:
// their branch metrics are the complements, so BX and BY swap roles (BM(~A, ~B) / 2 =
// Kc - BM(A, B) / 2, the identity BY = C - BX already rests on), the markers flipped unless mk.
__host__ __device__ constexpr int bx_src(int ph, int d) {
  if (d == 0) return -1;
  const uint32_t f = dw_flips(ph, d);
  for (int e = 0; e < d; e++) {
    const uint32_t fe = dw_flips(ph, e);
    if (ab_flips(f) == ab_flips(fe)) return e | (int)((((f ^ fe) >> 5) & 1u) << 8);
  }
#if ZRX_BX_COMP
  for (int e = 0; e < d; e++) {
    const uint32_t fe = dw_flips(ph, e);
    if ((ab_flips(f) ^ ab_flips(fe)) == 3) return e | (int)((((f ^ fe) >> 5) & 1u) << 8) | (1 << 9);
  }
#endif
  return -1;
}

// LDS byte address of a pointer into a __shared__ array (for inline-asm DS instructions)
__device__ __forceinline__ uint32_t lds_addr(const uint8_t* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)p;
}

// Per-lane constants (registers for the whole kernel; entries no column reads are dropped).
struct Consts {
  uint32_t sel[6][kDw];   // v_perm selector: per half [P byte of the state's (A, B)][its marker byte or 0]
  uint32_t sa[3];         // LDS ring byte offset of the lane's first position (dword 0, half 0) at C mod 6 = 0,2,4
};

__device__ __forceinline__ void make_consts(Consts& K, uint32_t l, uint32_t rib) {
#pragma unroll
  for (int ph = 0; ph < 6; ph++) {
#pragma unroll
    for (int d = 0; d < kDw; d++) {
      uint32_t s = 0;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t j = rotl6(pos_of(l, d, h), ph);
        const uint32_t bm = (j >> 5) & 1u;
        const uint32_t A = ((j >> 1) ^ (j >> 2) ^ (j >> 4)) & 1u;   // expected bits of j -> rotl6(j)
        const uint32_t B = (j ^ (j >> 1) ^ (j >> 2)) & 1u;          // (encoding.blk:92-109)
        s |= (bm ? 4u : 12u) << (16 * h);
        s |= (2u * A + B) << (16 * h + 8);
      }
      K.sel[ph][d] = s;
    }
  }
  // (the lane's other positions are at lane-uniform offsets from these: snap_delta)
#if defined(ZRX_EXPERIMENTS) && defined(ZRX_SNAP_SHARE)
  // (timing experiment, wrong output: rows 2 and 3 of each 32-lane half store their snapshots
  // over rows 0 and 1's, so no two rows of a half store to one bank at different addresses --
  // the snapshot stores' only bank conflicts -- with the same instructions and addresses in
  // bounds: does the kernel get faster without those conflicts?)
  rib &= ~2u;
#endif
#pragma unroll
  for (int k = 0; k < 3; k++) K.sa[k] = rib * 64u + rev6(rotl6(pos_of(l, 0, 0), 2 * k));
}
// ring-index offset of the position with in-lane bits (d, h) from the lane's first, at
// snapshot k (C mod 6 = 2k): position bit b -> state bit (b + 2k) mod 6 -> ring bit 5 - that
__host__ __device__ constexpr uint32_t snap_delta(int k, int d, int h) {
  const uint32_t p = (uint32_t)h | ((uint32_t)d << 1);
  uint32_t o = 0;
  for (int b = 0; b <= kDwBits; b++)
    if ((p >> b) & 1u) o |= 1u << (5 - (b + 2 * k) % 6);
  return o;
}

// Shift-free column (tests/vit8_model.py).  The column with cycle phase KPH = (c + 1) mod 8
// (c = the column computed; KPH 7 is the snapshot column) writes its marker at bit KPH of each
// half: a half is [0][H >> 1 in bits 14..8][the cycle's decisions in bits 7..0, oldest
// lowest].  Bits above the marker are still 0 in both candidates (cleared at KPH 0), so the
// marker breaks ties exactly like the brick's metric LSB (viterbicore.hpp:105-147), and the
// pads need no shift.  Branch metrics are added halved (BM / 2 at bit 8), so a half's sum
// (H >> 1) + BM / 2 <= 127 + 14 stays inside its 16 bits and a 32-bit add serves two halves;
// a wrap of the reference's u8 metric (H + BM > 255) sets bit 15, which the guarded column
// (G) clears after each add ("Guard-free columns": it never happens in the others).  A
// snapshot byte is bits 7..0 of a half as they are.
template <int PH, int KPH, int D, bool BYN = true>
__device__ __forceinline__ void column_bx(uint32_t (&BX)[kDw], uint32_t (&BY)[kDw], uint32_t P, const Consts& K,
                                          uint32_t C) {
  constexpr uint32_t mk = 1u << KPH;
  constexpr uint32_t mbits = mk * 0x00010001u;
  constexpr int src = bx_src(PH, D);
  // (a complement source needs its BY word, which pair phases do not compute: own v_perm then;
  // it happens only with 4-lane rows, whose pair phases have three dword bits)
  if constexpr (src < 0 || (((src >> 9) & 1) && !BYN)) {
    BX[D] = __builtin_amdgcn_perm(mk * 0x01010101u, P, K.sel[PH][D]);
  } else if constexpr ((src >> 9) & 1) {               // complement: the roles swap
    constexpr uint32_t fl = ((src >> 8) & 1) ? 0u : mbits;
    BX[D] = BY[src & 0xFF] ^ fl;
    BY[D] = BX[src & 0xFF] ^ fl;
    return;
  } else if constexpr ((src >> 8) == 0) {
    BX[D] = BX[src & 0xFF];
    if constexpr (BYN) BY[D] = BY[src & 0xFF];
    return;
  } else {
    BX[D] = BX[src & 0xFF] ^ mbits;
  }
  if constexpr (!BYN) return;
  // Keep C - BX a value of its own: reassociated as (partner T - BX) + C it would put two
  // adds after the AND on the column-to-column dependency chain instead of one.
  BY[D] = C - BX[D];
  asm("" : "+v"(BY[D]));
}
template <int PH, bool G, int D>
__device__ __forceinline__ void column_acs(uint32_t (&M)[kDw], const uint32_t (&T)[kDw], const uint32_t (&BX)[kDw],
                                           const uint32_t (&BY)[kDw]) {
  constexpr int pb = 5 - PH;                           // partner's position bit
  constexpr int src = bx_src(PH, D);
  uint32_t X, Z;
  if constexpr (pb == 0 && ((src >> 9) & 1) && !((src >> 8) & 1)) {
    // partner = the other half, words the complement of dword e's: the two halves of a word
    // then hold one branch metric and the two markers, so BX ^ markers is BX with its halves
    // swapped, and op_sel takes e's words as they are (no v_xor)
    constexpr int e = src & 0xFF;
    asm("v_pk_add_u16 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0]" : "=v"(X) : "v"(T[D]), "v"(BY[e]));
    asm("v_pk_add_u16 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0]" : "=v"(Z) : "v"(T[D]), "v"(BX[e]));
  } else if constexpr (pb == 0) {  // partner = the other half: [T.lo + BY.hi][T.hi + BY.lo] in one op
    X = T[D] + BX[D];
    asm("v_pk_add_u16 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1]" : "=v"(Z) : "v"(T[D]), "v"(BY[D]));
  } else if constexpr (pb <= kDwBits) {                // partner = another dword of the lane
    X = T[D] + BX[D];
    Z = T[D ^ (1 << (pb - 1))] + BY[D];
  } else {                                             // partner lane: the DPP source of the add
    X = T[D] + BX[D];
    Z = (uint32_t)__builtin_amdgcn_mov_dpp((int)T[D], partner_dpp(pb), 0xF, 0xF, true) + BY[D];
  }
  if constexpr (G) {                                   // the u8 wrap (bit 15 of a half)
    X &= 0x7FFF7FFFu;
    Z &= 0x7FFF7FFFu;
  }
  M[D] = w32(__builtin_elementwise_min(h2(X), h2(Z)));
}
// G: wrap the metrics mod 256 after every add (two ANDs per dword).  Without it (G false)
// the column has no AND except at KPH 0, which clears the cycle's history: see "Guard-free
// columns" below.
// Phases whose partner is another dword of the lane: the two dwords form butterflies with the
// same branch-metric words (the partner's BX is BX with the markers flipped), and
// S = T[D] + T[D'] + C serves both: T[D'] + (C - BX) = S - (T[D] + BX), so the pair needs one
// add3 instead of two C - BX subtractions.  The 32-bit sums are the same integers as T' + BY
// (carries between the halves cancel), so the result is bit-identical.
template <int PH, bool G, int D>
__device__ __forceinline__ void column_pair(uint32_t (&M)[kDw], const uint32_t (&T)[kDw], const uint32_t (&BX)[kDw],
                                            uint32_t C) {
  constexpr int Dp = D ^ (1 << (5 - PH - 1));
  if constexpr (D < Dp) {
    uint32_t S = T[D] + T[Dp] + C;
    asm("" : "+v"(S));                                 // (else S - X folds back into T[D'] + C - BX)
    uint32_t X = T[D] + BX[D], Xp = T[Dp] + BX[Dp];
    uint32_t Z = S - X, Zp = S - Xp;
    if constexpr (G) {
      X &= 0x7FFF7FFFu;
      Z &= 0x7FFF7FFFu;
      Xp &= 0x7FFF7FFFu;
      Zp &= 0x7FFF7FFFu;
    }
    M[D] = w32(__builtin_elementwise_min(h2(X), h2(Z)));
    M[Dp] = w32(__builtin_elementwise_min(h2(Xp), h2(Zp)));
  }
}
#ifndef ZRX_PAIR_S
#define ZRX_PAIR_S 1
#endif
template <int PH, int KIND, int KPH, bool G, int... D>
__device__ __forceinline__ void column5_(uint32_t (&M)[kDw], uint32_t P, const Consts& K, std::integer_sequence<int, D...>) {
  const uint32_t T[kDw] = {(KPH == 0 ? (M[D] & 0x7F007F00u) : M[D])...};
  constexpr uint32_t mk = 1u << KPH;
  constexpr uint32_t Kc = KIND == 0 ? 14u : 7u;        // (28 or 14) / 2: a column's complementary BM / 2
  constexpr uint32_t C = ((Kc << 8) | mk) * 0x00010001u;
  constexpr int pb = 5 - PH;
  uint32_t BX[kDw], BY[kDw];
  if constexpr (ZRX_PAIR_S && pb >= 1 && pb <= kDwBits) {
    (column_bx<PH, KPH, D, false>(BX, BY, P, K, C), ...);
    (column_pair<PH, G, D>(M, T, BX, C), ...);
  } else {
    (column_bx<PH, KPH, D>(BX, BY, P, K, C), ...);
    (column_acs<PH, G, D>(M, T, BX, BY), ...);
  }
}
template <int PH, int KIND, int KPH, bool G = true>
__device__ __forceinline__ void column5(uint32_t (&M)[kDw], uint32_t P, const Consts& K) {
  column5_<PH, KIND, KPH, G>(M, P, K, std::make_integer_sequence<int, kDw>{});
}

// ---- Guard-free columns -------------------------------------------------------------------
// The guard exists for one event: H + BM passing 255 (the brick's u8 metric wraps), which
// sets bit 15 of a half; the guarded column clears it after each add (two ANDs per dword).
// Without wraps there is nothing to clear.  When can a wrap happen?  H is exact integer
// arithmetic until the first wrap, bounded by:
//  * H_min never decreases from column to column (all branch metrics are >= 0) and grows by at
//    most 14 per full column and 7 per punctured one (a state's two successors differ in both
//    coded bits, so their branch metrics sum to 28 / 14);
//  * every state is reached from any state 6 columns earlier (K = 7), so
//    H_max(t) <= H_min(t - 6) + P6 with P6 the largest branch-metric sum of 6 columns:
//    168 at rate 1/2, 126 at 2/3 (3 full + 3 punctured), 112 at 3/4 (2 full + 4 punctured);
//  * normalize subtracts H_min, which is >= H_min 6 columns earlier.
// Rates 1/2 and 2/3 normalize every 8 columns, so H_min(t - 6) <= 14 in the current
// normalization's units and H_max + BM <= 14 + 168 + 28 = 210 (the initial 0 / 48 metrics:
// <= 48 + 5 x 28 + 28 = 216): they never wrap, and run guard-free always.  Rate 3/4
// normalizes every 24 columns (one body), where the bound allows a wrap late in a body once
// H_min passes 115.  So a rate-3/4 body runs guard-free speculatively and checks H_min at its
// columns 6, 12 and 18: if every check finds a state with H <= 115 (a row's H_min <= 115),
// then for every column t + 1 of the body H_max(t) <= H_min(c) + 112 <= 227 with c the check
// at or after t - 6 (columns 0..5 use the previous body, H_min <= 0 after its normalize), so
// no add wrapped (induction over t) and the body is exact (half < 58 << 8: H >> 1 <= 57).  Otherwise the wave redoes the body
// from its saved metrics with the guard (config 3 never does: its H stays below 84).  Bodies
// with events run speculatively as well: the row state (Row, its RowX entry, s_next) is saved
// with the metrics, and a body with a deferred traceback walk is redone without the walk.  Each
// check is one 16-bit compare of one half per lane (any state <= 115 suffices) and a ballot.
#ifndef ZRX_NOGUARD
#define ZRX_NOGUARD 1
#endif
constexpr bool kNoGuard = ZRX_NOGUARD != 0;
// every row (kLanes-bit group) of a lane mask has a bit set
__device__ __forceinline__ bool rows_all_any(uint64_t m) {
  if constexpr (kLanes == 8) {
    return ((m - 0x0101010101010101ull) & ~m & 0x8080808080808080ull) == 0ull;
  } else {
    bool ok = true;
#pragma unroll
    for (int r = 0; r < kRowsWave; r++) ok = ok && ((m >> (r * kLanes)) & kRowMask) != 0ull;
    return ok;
  }
}

// normalize (viterbicore.hpp:149-168): H -= min over the row's 64 H bytes (H even).
__device__ __forceinline__ void normalize(uint32_t (&M)[kDw]) {
  u16x2 t = h2(M[0]);
#pragma unroll
  for (int d = 1; d < kDw; d++) t = __builtin_elementwise_min(t, h2(M[d]));
  uint32_t v = (uint32_t)min(t.x, t.y);
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));
  if constexpr (kLanes >= 8) v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));
  if constexpr (kLanes == 16) v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false));
  const uint32_t rep = __builtin_amdgcn_perm(0u, v, 0x010C010Cu);   // [H][0][H][0]
#pragma unroll
  for (int d = 0; d < kDw; d++) M[d] = w32(h2(M[d]) - h2(rep));
}
// min / max of a row-uniform value over the wave's rows (scalar)
__device__ __forceinline__ uint32_t wave_min_rows(uint32_t v) {
  uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
#pragma unroll
  for (int r = 1; r < kRowsWave; r++) m = min(m, (uint32_t)__builtin_amdgcn_readlane((int)v, r * kLanes));
  return m;
}

// 64-bit value of `lane` as a wave-uniform scalar
__device__ __forceinline__ int64_t rl64(int64_t v, int lane) {
  return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), lane) << 32) |
                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane));
}
constexpr int64_t kSoftWindow = 0xFFFFFF00;

// ZRX_GUARD builds (debugging only, scripts/build_guard.sh): every global store of the
// Viterbi is range-checked against the output buffer the host registered, and a violation
// is printed and skipped instead of faulting.
#ifdef ZRX_GUARD
__device__ uint64_t g_zg_out_lo, g_zg_out_hi;
__device__ uint32_t g_zg_np;
#define ZG_OUT_BAD(lo, hi) ((uint64_t)(uintptr_t)(lo) < g_zg_out_lo || (uint64_t)(uintptr_t)(hi) > g_zg_out_hi)
#else
#define ZG_OUT_BAD(lo, hi) false
#endif           // span of one buffer window over soft values

// Rate tables: steps per group, soft values per group, soft values per 24-column body.
template <int CR> struct Rate;
template <> struct Rate<0> { static constexpr int steps = 1, G = 2, chunk = 48; };   // 1/2
template <> struct Rate<1> { static constexpr int steps = 2, G = 3, chunk = 36; };   // 2/3
template <> struct Rate<2> { static constexpr int steps = 3, G = 4, chunk = 32; };   // 3/4

// ---- Trellis segments -------------------------------------------------------------------
// A long frame is decoded as nseg segments side by side (rows of their own), so a batch of
// few or unequal frames still fills every SIMD.  Segment k >= 1 starts at column
// S_k = 768 m_k (768 = lcm of the 24-column body and the 256-bit window) from all-zero
// metrics and owns the output windows from J_k = S_k + 256 on; segment k - 1 runs on until
// it has written the window ending at J_k (the window at ob = J_k - 256 fires at the first
// group end with tr >= J_k + 30).  The future of the brick loop depends on the column, the
// window schedule (ob) and the even parts H of the 64 metrics only (viterbicore.hpp:105-168:
// the marker LSB is masked off before every add, normalize subtracts min & 0xFE), and the
// tracebacks of windows from J_k on read decisions of columns > J_k only.  So if both
// segments hold the same normalized H vector at the seam column C_k = S_k + 240 (a body end,
// after 240 warm-up columns), every output bit of segment k equals the unsplit decode's.
// Both sides store their metrics at C_k (the seam "dumps"); a second pass (fix) compares
// them and, for the first seam of a frame that disagrees, re-decodes from C_k with segment
// k - 1's exact register state, until it agrees with a later segment's start state (or to
// the frame's end).  Bit-exact either way; warm-up from zero converges in < 100 columns on
// every chain input measured, so the fix pass normally finds nothing to do.
constexpr uint32_t kSegUnit = 768;
// Warm-up W = J_k - S_k, and C_k = S_k + W - 16 (the last body end before J_k).  J_k = 768 m_k
// + 256 whatever W is, so W = 16 mod 24 keeps S_k a multiple of 24.  A uniform batch's rows are
// placed so that every wave holds one segment index k (viterbi_rows), so its waves' windows
// stay aligned with any W and it warms up for 136 columns: soft values from the chain converge
// within 72 columns at AWGN sigma 4..12 and within 120 at sigma 58, where CRCs start to fail
// (warm-ups from zero at every 768th column of config-3 packets, 420 per sigma, brick loop in
// numpy), and 120 columns fewer per seam than 256 take 7.5 % off a 2048-packet shard's longest
// row.  A mixed batch's segments of one packet share a wave with segment 0, whose windows sit at
// multiples of 256: it keeps W = 256.
constexpr uint32_t kSegWarm = 256;                     // S_k -> J_k (mixed batches)
constexpr uint32_t kSegWarmUni = 136;                  // S_k -> J_k (uniform batches)
static_assert(kSegWarm % 24 == 16 && kSegWarmUni % 24 == 16, "S_k = J_k - W must stay a multiple of 24");
__host__ __device__ constexpr uint32_t seg_cmp(uint32_t warm) { return warm - 16u; }   // S_k -> C_k
constexpr uint32_t kSegCmp = seg_cmp(kSegWarm);
constexpr int kMaxSeg = 8;
constexpr uint32_t kMinSeg = 1536;                     // columns per segment at least (mixed batch)
// A uniform batch too small to give every SIMD two waves of whole frames is cut into segments
// of at least kMinCut columns: a 2048-packet config-3 shard (a config-4 rank at N = 8) then
// takes 8 segments of 2 units (16384 rows, two waves per SIMD) instead of 7 of 2-3 units,
// whose longest row (3 units + the seam overlap) set the kernel's time.
constexpr uint32_t kMinCut = 1024;
constexpr uint32_t kSegMaxEnd = 1u << 24;              // longer frames are not split
constexpr uint32_t kSeamWords = 32;                    // uint2 per dump slot (kLanes x kDw / 2 used: 16)
// Segment length of a mixed batch: L x kSegMixNum / 8, L = the batch's columns / (64 rows
// per CU); the launch grid allows 8 / kSegMixNum x 64 rows per CU + one per packet.
// Measured on config 5 (interleaved A/B, 3 rounds): 4/8 L 0.62 ms Viterbi, 6/8 0.585, 8/8
// 0.584, 9/8 0.578, 11/8 0.570, 14/8 0.622 — shorter segments pay more seam overlap than
// they save in tail, longer ones leave rows above the batch's fair share.
#ifndef ZRX_SEG_MIX_NUM
#define ZRX_SEG_MIX_NUM 11
#endif
constexpr uint32_t kSegMixNum = ZRX_SEG_MIX_NUM;

// floor(y / n) for n = 1..8 and y < 2^20 by a reciprocal multiply (exact there: the error
// term y / 2^32 stays below the 1/8 gap to the next integer)
__host__ __device__ __forceinline__ uint32_t udiv_small(uint32_t y, uint32_t n) {
  return n <= 1u ? y : (uint32_t)(((uint64_t)y * (0xFFFFFFFFu / n + 1u)) >> 32);
}
// floor(b / d) for b < 2^20 and 2 <= d < 4096 with rcp = 0xFFFFFFFF / d + 1 (exact: the
// error term b / 2^32 stays below the 1 / d gap to the next integer)
__host__ __device__ __forceinline__ uint32_t udiv_rcp(uint32_t b, uint32_t rcp) {
  return (uint32_t)(((uint64_t)b * rcp) >> 32);
}
// Sorted position -> row slot: the nfull whole blocks of kRows rows placed "snake" over ncu
// CUs: in odd rounds of ncu blocks the order is reversed, so with blocks dealt to CU
// (slot mod ncu) — what the dispatcher does when every block of the launch is resident
// (scripts/ubench/hwid.hip) — the CU running one of the longest blocks gets one of the
// shortest of the next round beside it.  An involution within each round; a partial last
// block stays in place.  rcp = 0xFFFFFFFF / ncu + 1 (ncu >= 2).
__host__ __device__ __forceinline__ uint32_t order_place(uint32_t pos, uint32_t nfull, uint32_t ncu, uint32_t rcp) {
  const uint32_t b = pos / (uint32_t)kRows;
  if (b >= nfull) return pos;
  const uint32_t r = udiv_rcp(b, rcp), c = b - r * ncu, base = r * ncu;
  const uint32_t m = min(ncu, nfull - base);
  return ((r & 1u) ? base + m - 1u - c : b) * (uint32_t)kRows + pos % (uint32_t)kRows;
}
// A mixed batch's whole blocks ranked by their longest row (0 = longest; plan_rows_mixed)
// -> block slot, for blocks dealt to CU slot mod ncu.  Up to two rounds: the longest blocks
// alone on the CUs the second round leaves free (the shortest of them on the CU that also
// gets the partial last block, slot nfull), the rest paired longest with shortest.  More
// rounds: the snake of order_place over the ranks.  A permutation of 0 .. nfull - 1.
constexpr int kRankBlocks = 8192;                      // ranked when the batch has at most this many
__host__ __device__ __forceinline__ uint32_t rank_place(uint32_t r, uint32_t nfull, uint32_t ncu, uint32_t rcp) {
  if (nfull <= ncu) return r;
  if (nfull <= 2u * ncu) {
    const uint32_t n2 = nfull - ncu, alone = ncu - n2;   // CUs with two whole blocks, with one
    if (r < alone) return ncu - 1u - r;
    const uint32_t q = r - alone;                      // CU c: ranks alone + c and alone + 2 n2 - 1 - c
    return q < n2 ? q : ncu + (2u * n2 - 1u - q);
  }
  return order_place(r * (uint32_t)kRows, nfull, ncu, rcp) / (uint32_t)kRows;
}
// The plan header k_pkt_plan writes for k_viterbi3 (int32 words of the nrows buffer).
// Words 8..13: the uniform batch the arrays of the last rx-chain plan describe (kPlanExpN
// packets, 0 = none, of these {frame_len, code_rate, soft_len, modulation}) and the flag
// k_signal_vit raises when a packet of a batch of that size asks for something else: a
// batch equal in all of it reuses the plan (k_pkt_plan returns at once).
enum PlanWord { kPlanRows = 0, kPlanFixes = 1, kPlanUniform = 2, kPlanNcu = 3, kPlanSegLen = 4, kPlanDropped = 5,
                kPlanExpN = 8, kPlanExpLen = 9, kPlanExpCr = 10, kPlanExpSoft = 11, kPlanExpMod = 12,
                kPlanMismatch = 13, kPlanWords = 16 };
constexpr int kPlanUnit = kRows;                       // rows ranked together by the mixed plan (a block's)

// start unit m_k of segment k >= 1 of nseg over a frame of E = 8 len + 6 columns (rounded
// k E / nseg; with E / nseg >= kMinCut the m_k are distinct (steps of > 1 unit) and
// S_k + 256 + 64 <= E (the last start is at most (nseg - 1) E / nseg + 384))
__host__ __device__ __forceinline__ uint32_t seg_start(uint32_t E, uint32_t nseg, uint32_t k, uint32_t warm = kSegWarm) {
  // floor(x / (1536 nseg)) = floor(floor(x / 1536) / nseg)
  return k == 0 ? 0u : kSegUnit * udiv_small((2u * k * E + nseg * kSegUnit) / (2u * kSegUnit), nseg) + kSegWarm - warm;
}
// segments for a frame of E columns with cols columns of input, target length L, segments of
// at least min_len (kMinSeg or kMinCut) columns
__host__ __device__ __forceinline__ uint32_t seg_count(uint32_t E, uint32_t cols, uint32_t L,
                                                       uint32_t min_len = kMinSeg) {
  if (cols < E || E > kSegMaxEnd || E < 2u * min_len || L == 0) return 1u;
  uint32_t n = (cols + L - 1u) / L;
  n = min(n, E / min_len);
  return min(max(n, 1u), (uint32_t)kMaxSeg);
}
// first column after segment k (absolute): where segment k + 1's first window is written
__host__ __device__ __forceinline__ uint32_t seg_stop(uint32_t E, uint32_t cols, uint32_t nseg, uint32_t k,
                                                      uint32_t warm = kSegWarm) {
  return k + 1u < nseg ? seg_start(E, nseg, k + 1u, warm) + warm + 30u : cols;
}
// dump of seam j (1 <= j < nseg) of packet p, side 0 (segment j - 1) or 1 (segment j)
__host__ __device__ __forceinline__ size_t seam_index(uint32_t p, uint32_t j, uint32_t side) {
  return (((size_t)p * (kMaxSeg - 1) + (j - 1u)) * 2u + side) * kSeamWords;
}

// Cold per-row facts for the seam events, one entry per row of the block (LDS).
struct RowX {
  uint32_t p;                                          // packet
  uint32_t kn;                                         // k | nseg << 8 | fix << 16 | matched << 17 | short warm-up << 18 | seam j << 20
  uint32_t S, E;                                       // first column (absolute), 8 len + 6
};

// Per-row decoder state (row-uniform values in VGPRs).  Columns are relative to the row's
// first column S (a multiple of 24, so body phases are the frame's own).
struct Row {
  uint32_t ob, end, cols, next;       // output bits so far, 8*frame_len+6, columns of input, next event column
  uint32_t evc;                       // next seam event column (kNever: none)
  bool live;                          // still decoding (not done, input not exhausted)
  bool ppend, fpend;                  // partial / final traceback due at the body end
  uint32_t pT, plook, fT, fcnt, flook;
  uint32_t pM[kDw], fM[kDw];
  uint32_t nbytes;                    // bytes written so far
};

__device__ __forceinline__ uint32_t row_next(const Row& R) {
  if (!R.live) return kNever;
  return min(min(R.ob + 286u, R.end), min(R.cols, R.evc));
}
// the lanes of this lane's row in a wave ballot, shifted down to bit 0
__device__ __forceinline__ uint32_t row_bits(uint64_t ballot) {
  return (uint32_t)(ballot >> (__lane_id() & (64u - kLanes))) & kRowMask;
}
// a seam dump: the row's 64 metric halves, kDw / 2 uint2 per lane
__device__ __forceinline__ void dump_store(uint2* __restrict__ at, uint32_t l, const uint32_t (&M)[kDw]) {
#pragma unroll
  for (int i = 0; i < kDw / 2; i++) at[(kDw / 2) * l + i] = make_uint2(M[2 * i], M[2 * i + 1]);
}
__device__ __forceinline__ void dump_load(const uint2* __restrict__ at, uint32_t l, uint32_t (&M)[kDw]) {
#pragma unroll
  for (int i = 0; i < kDw / 2; i++) {
    const uint2 v = at[(kDw / 2) * l + i];
    M[2 * i] = v.x; M[2 * i + 1] = v.y;
  }
}
// do the H bits (& 0x7F007F00) of two dumps differ in this lane?
__device__ __forceinline__ bool dump_ne(const uint2* __restrict__ a, const uint2* __restrict__ b, uint32_t l) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < kDw / 2; i++) {
    const uint2 u = a[(kDw / 2) * l + i], v = b[(kDw / 2) * l + i];
    x |= (u.x ^ v.x) | (u.y ^ v.y);
  }
  return (x & 0x7F007F00u) != 0u;
}

// Seam event of a row at relative column tr (a body end, after normalize): a segment stores
// its metrics for the fix pass; a fix row compares its own with the next segment's start
// state and, when they agree, stops where that segment's windows begin.
__device__ __forceinline__ void seam_event(Row& R, uint32_t tr, const uint32_t (&M)[kDw], uint32_t l, uint32_t rib,
                                        RowX* rowx, uint2* __restrict__ dumps) {
  RowX x = rowx[rib];
  const uint32_t k = x.kn & 0xFFu, nseg = (x.kn >> 8) & 0xFFu, fix = (x.kn >> 16) & 1u, j = x.kn >> 20;
  const uint32_t W = (x.kn >> 18) & 1u ? kSegWarmUni : kSegWarm;
  (void)tr;
#ifdef ZRX_GUARD
  if (x.p >= g_zg_np || j == 0 || j >= nseg || nseg > (uint32_t)kMaxSeg) {
    printf("ZG seam_event bad: blk %d rib %u p %u k %u nseg %u fix %u j %u tr %u S %u E %u\n", (int)blockIdx.x, rib, x.p,
           k, nseg, fix, j, tr, x.S, x.E);
    R.evc = kNever;
    return;
  }
#endif
  if (!fix) {
    const uint32_t side = j == k ? 1u : 0u;            // at C_k: segment k's start; at C_{k+1}: its end side
    dump_store(dumps + seam_index(x.p, j, side), l, M);
    if (side == 1u && k + 1u < nseg) {
      x.kn = (x.kn & 0xFFFFFu) | ((k + 1u) << 20);
      R.evc = seg_start(x.E, nseg, k + 1u, W) + seg_cmp(W) - x.S;
    } else {
      R.evc = kNever;
    }
  } else {
    uint32_t B[kDw];
    dump_load(dumps + seam_index(x.p, j, 1u), l, B);
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < kDw; i++) d |= M[i] ^ B[i];
    const uint64_t bad = __builtin_amdgcn_ballot_w64((d & 0x7F007F00u) != 0u);
    if (row_bits(bad) == 0u) {                         // the row's 64 H bytes agree
      R.cols = min(R.cols, seg_start(x.E, nseg, j, W) + W + 30u - x.S);
      x.kn |= 1u << 17;
      R.evc = kNever;
    } else if (j + 1u < nseg) {
      x.kn = (x.kn & 0xFFFFFu) | ((j + 1u) << 20);
      R.evc = seg_start(x.E, nseg, j + 1u, W) + seg_cmp(W) - x.S;
    } else {
      R.evc = kNever;
    }
  }
  rowx[rib] = x;
}

// Events after a group ending at column tr (sora_ext_viterbi.cpp:112-149); normalize ran first.
// (Reads no LDS ring slot: see the snapshot-store invariant at Packet::ds_b8_hi.)
__device__ __forceinline__ void events(Row& R, uint32_t tr, const uint32_t (&M)[kDw]) {
  if (R.live && tr >= R.next) {
    if (tr >= R.end) {                                  // final traceback
      R.fpend = true; R.fT = tr;
#pragma unroll
      for (int d = 0; d < kDw; d++) R.fM[d] = M[d];
      R.fcnt = R.end - R.ob - 6u; R.flook = tr - R.end;
      R.live = false;
    } else if (tr >= R.ob + 286u) {                     // 256 bits, lookahead 24 + (tr-thresh)%8
      R.ppend = true; R.pT = tr;
#pragma unroll
      for (int d = 0; d < kDw; d++) R.pM[d] = M[d];
      R.plook = 24u + ((tr - (R.ob + 286u)) & 7u);
      R.ob += 256u;
    }
    if (tr >= R.cols) R.live = false;                   // input exhausted: no more groups
    R.next = row_next(R);
  }
}

// A traceback walk shared by the rows of a wave (same window), deferred to the next body:
// its nl + 32 steps (nl lookahead blocks, then the window's 32 output bytes, newest first)
// run inside that body's columns, two per column in columns 0..11 and one per column after
// (Packet::walk_col), so each step's LDS latency hides behind column work.  A step packs the
// byte read before into a dword, moves the ring index on and issues the next read; every
// fourth output byte stores the dword with a buffer store (rows that do not own the window
// store out of range, i.e. nothing).  The slot base steps back on the scalar unit.
// we = nl (0: nothing deferred).
struct Walk {
  int we;                         // wave-uniform
  uint32_t A;                     // wave-uniform: slot of the pending read
  uint32_t ix, b, acc, voff;      // per lane: ring index (row offset included), pending byte, dword, store offset
  uint64_t ob;                    // wave-uniform: output base the store offsets are relative to
};
// (The base is re-read as wave-uniform here: built from the struct field as it is, the
// descriptor was not provably uniform across the body's control flow, and every store became
// a waterfall loop of readfirstlanes, 64-bit compares and exec updates.)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t walk_rsrc(const Walk& W) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)W.ob);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(W.ob >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, 0x7FFFFFFF, 0x00020000);
}
// The setup runs in a branch whose join the divergence analysis cannot prove uniform; the
// scalar fields are uniform by construction, so they are re-read as such.
__device__ __forceinline__ void walk_uniform(Walk& W) {
  W.we = __builtin_amdgcn_readfirstlane(W.we);
  W.A = (uint32_t)__builtin_amdgcn_readfirstlane((int)W.A);
  W.ob = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(W.ob >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)W.ob);
}

// One walk step t (compile-time when called from the body columns).
template <bool FAKE = false, class I>
__device__ __forceinline__ void walk_stepk(Walk& W, I t, uint32_t nl, const uint8_t* ring0, uint32_t rb) {
  constexpr uint32_t span = (uint32_t)kRing * kSlotBytes;
  const uint32_t b = W.b;
  W.acc = (W.acc << 8) | b;                            // lookahead bytes leave before the first store
  W.ix = (b & 63u) | rb;
  W.A = W.A == 0u ? span - (uint32_t)kSlotBytes : W.A - (uint32_t)kSlotBytes;
  if constexpr (FAKE) {                                // (timing experiment: no LDS read on the chain)
    if (t + 1 < nl + 32u) W.b = (W.ix * 5u + W.A) & 0xFFu;
  } else {
    if (t + 1 < nl + 32u) W.b = ring0[W.A + W.ix];
  }
  if (t >= nl && ((t - nl) & 3u) == 3u)                // output bytes 31-o .. 34-o, o = t - nl
    __builtin_amdgcn_raw_buffer_store_b32(W.acc, walk_rsrc(W), (int)(W.voff + 31u - (t - nl)), 0, 0);
}
// The deferred walk without a following body (the rows stopped): its steps back to back.
__device__ __forceinline__ void walk_finish(Walk& W, const uint8_t* ring0, uint32_t rb) {
  const uint32_t nl = (uint32_t)W.we;
  for (uint32_t t = 0; t < nl + 32u; t++) walk_stepk(W, t, nl, ring0, rb);
  W.we = 0;
}

// Traceback of one window for the rows with `due` set: argmin over the row (all lanes),
// then one lane per row walks the snapshot ring and writes the window's bytes.  The walk is
// a chain of dependent LDS reads (state -> byte -> state 8 columns back), so the loop body
// keeps only the read, the bit reversal and the address add on that chain.
// DEFER (partial windows): rows sharing a window leave the window's last 24 or 16 output
// bytes to the next body's columns (W); tr0 is the first column of the body that raised the
// event.
template <bool DEFER = false>
__device__ __forceinline__ void traceback(bool due, const uint32_t (&M)[kDw], uint32_t T, uint32_t cnt,
                                          uint32_t look, uint32_t l, uint32_t rib, const uint8_t* ring,
                                          uint8_t* __restrict__ out, uint32_t ooff, uint32_t& nbytes,
                                          Walk* W = nullptr, uint32_t tr0 = 0) {
  const uint32_t ph = T % 6u;
  // H in bits 14..8 (halved), the marker of column T at bit (T+1)%8; the n = (T-6)%8 newest
  // decisions in bits n-1..0
  const uint32_t n = (T - 6u) & 7u, ms = (T + 1u) & 7u;
  // the state of half q: pos_of(l, q >> 1, q & 1) = pos_of(l, 0, 0) ^ q, and rotl6 is linear
  // over XOR, so st(q) = rotl6(pos_of(l, 0, 0), ph) ^ rotl6(q, ph)
  // rotl6(x, ph) = bits 6 - ph .. 11 - ph of (x x) = 65 x: one shift of the doubled label
  const uint32_t o = 6u - ph;
  const uint32_t st0 = ((pos_of(l, 0, 0) * 65u) >> o) & 63u;
  const uint32_t r0 = (65u >> o) & 63u, r1 = (130u >> o) & 63u, r2 = (260u >> o) & 63u;
  uint32_t s0, pad;
  bool walker;
  uint64_t wm;
  if constexpr (kDw == 4) {
    // 16-bit keys, both halves of a dword at once: [H bits 7..1][marker][st][0 0], in signed
    // int16 order (the 32-bit key below without its pad byte; st is unique in the row, so
    // the pad never decides).  The winner's pad is then read from the lane that holds it.
    const uint32_t sh = 8u - ms;                       // marker bit ms -> bit 8 of each half
    const uint32_t c0 = (st0 << 2) | ((st0 ^ r0) << 18);   // st of halves (2d, 2d + 1), at bits 2, 18
    const uint32_t rr1 = r1 * 0x40004u, rr2 = r2 * 0x40004u;
    const uint32_t stc[4] = {c0, c0 ^ rr1, c0 ^ rr2, c0 ^ rr1 ^ rr2};
    i16x2 acc;
#pragma unroll
    for (int d = 0; d < 4; d++) {
      const uint32_t y = ((M[d] << sh) & 0x01000100u) | stc[d];
      const i16x2 k = __builtin_bit_cast(i16x2, ((M[d] << 1) & 0xFE00FE00u) | y);
      acc = d == 0 ? k : __builtin_elementwise_min(acc, k);
    }
    int32_t kb = min((int32_t)acc.x, (int32_t)acc.y);
    kb = min(kb, __builtin_amdgcn_update_dpp(0, kb, 0xB1, 0xF, 0xF, false));
    kb = min(kb, __builtin_amdgcn_update_dpp(0, kb, 0x4E, 0xF, 0xF, false));
    kb = min(kb, __builtin_amdgcn_update_dpp(0, kb, 0x141, 0xF, 0xF, false));
    walker = due && l == 0 && cnt != 0;
    wm = __builtin_amdgcn_ballot_w64(walker);
    if (wm == 0) return;
    s0 = ((uint32_t)kb >> 2) & 63u;
    // the winner's half q in its lane: q = rotr6(s0 ^ st0, ph) < 8 (position bits 0..2);
    // the row's 8 pad bytes in byte order q, one v_perm picks it, the other lanes give 0
    const uint32_t x = (s0 ^ st0) * 65u;               // (x x): rotr6 is one bit-field extract
    const uint32_t q = (x >> ph) & 63u;
    const uint32_t pk0 = __builtin_amdgcn_perm(M[1], M[0], 0x06040200u);
    const uint32_t pk1 = __builtin_amdgcn_perm(M[3], M[2], 0x06040200u);
    const uint32_t in_lane = (uint32_t)((int32_t)(q - 8u) >> 31);
    uint32_t pb = __builtin_amdgcn_perm(pk1, pk0, q) & in_lane & 0xFFu;
    pb |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pb, 0xB1, 0xF, 0xF, false);
    pb |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pb, 0x4E, 0xF, 0xF, false);
    pb |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pb, 0x141, 0xF, 0xF, false);
    pad = (pb << (8u - n)) & 0xFFu;                    // as the shifted pad: newest at bit 7
  } else {
    uint32_t best = 0xFFFFFFFFu;
#pragma unroll
    for (int q = 0; q < 2 * kDw; q++) {
      const uint32_t half = M[q >> 1] >> (16 * (q & 1)) & 0xFFFFu;
      const uint32_t st = st0 ^ ((q & 1) ? r0 : 0u) ^ ((q & 2) ? r1 : 0u) ^ ((q & 4) ? r2 : 0u) ^
                          ((q & 8) ? (520u >> o) & 63u : 0u);
      const uint32_t pd = ((half & ((1u << n) - 1u)) << (8u - n)) & 0xFFu;   // as the shifted pad: newest at bit 7
      // the key (m << 8 | 4 st) in signed int16 order, m = H | marker, above the pad:
      // [H bits 7..1 ^ sign][marker][st][0 0][pad]
      const uint32_t key = (((half & 0x7F00u) << 17) | (((half >> ms) & 1u) << 24) | (st << 18) | pd) ^ 0x80000000u;
      best = min(best, key);
    }
    best = min(best, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)best, 0xB1, 0xF, 0xF, false));
    best = min(best, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)best, 0x4E, 0xF, 0xF, false));
    if constexpr (kLanes >= 8) best = min(best, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)best, 0x141, 0xF, 0xF, false));
    if constexpr (kLanes == 16) best = min(best, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)best, 0x140, 0xF, 0xF, false));
    walker = due && l == 0 && cnt != 0;
    wm = __builtin_amdgcn_ballot_w64(walker);
    if (wm == 0) return;
    s0 = (best >> 18) & 63u;
    pad = best & 0xFFu;
  }
  // bit i of Z = decision of column T + 6 - i along the best path (state bits, then the pad)
  const uint32_t Z = s0 | ((__builtin_bitreverse32(pad) >> 24) << 6);
  const uint32_t C0 = T - ((T - 6u) & 7u);             // newest snapshot column <= T
  const uint32_t c_hi = T - look;
  const uint32_t nlook = (C0 - c_hi) >> 3, nout = cnt >> 3;
  constexpr uint32_t span = (uint32_t)kRing * kSlotBytes;
  // Do the walking rows share their window (C0, c_hi, nout)?  Then the slot sequence is
  // wave-uniform: the slot base steps back on the scalar unit and a walk step is one
  // v_and_or (next ring index) plus the LDS address add.  (Always the case for a batch of
  // equal packets; mixed rows take the per-row walk below.)
  const int first = (int)__builtin_ctzll(wm);
  const uint32_t C0f = (uint32_t)__builtin_amdgcn_readlane((int)C0, first);
  const uint32_t chf = (uint32_t)__builtin_amdgcn_readlane((int)c_hi, first);
  const uint32_t nof = (uint32_t)__builtin_amdgcn_readlane((int)nout, first);
  const uint64_t ob_me = (uint64_t)(uintptr_t)out;    // rows of one window share the 4 GiB output base
  const uint64_t obf = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(ob_me >> 32), first) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ob_me, first);
  const bool uni = __builtin_amdgcn_ballot_w64(walker && (C0 != C0f || c_hi != chf || nout != nof ||
                                                          ob_me != obf)) == 0;
  const uint32_t rb = rib * 64u;
  uint32_t ix = rb + (__builtin_bitreverse32((Z >> (T - C0)) & 63u) >> 26);   // ring index = rev6(state)
  // Deferral: window step i reads slot C0 - i.  The next body's snapshot k (k = 0, 1, 2, at
  // the end of its column 5 + 8k) overwrites slot C0 - (38 - k - s), s = slots between C0
  // and this body's newest snapshot (tr0 + 22).  With two steps per column in columns 0..11
  // and one after, the read of step i is issued in column i / 2 (i <= 24) or i - 12: before
  // every overwrite of a window slot when s <= 2 (s = 3 only occurs with T in a body's first
  // six columns; those windows walk now).
  const uint32_t s = (tr0 + 22u - C0f) >> 3;
  const uint32_t nlf = (C0f - chf) >> 3;
  uint8_t* op = out + ooff + ((c_hi - 14u) >> 3);      // output byte of block c_hi, newest first
  auto prevS = [](uint32_t x) { return x == 0u ? span - (uint32_t)kSlotBytes : x - (uint32_t)kSlotBytes; };
#ifdef ZRX_GUARD
  if (walker && ZG_OUT_BAD(op + 1 - (int)nout, op + 1)) {
    printf("ZG traceback bad: blk %d rib %u T %u cnt %u look %u c_hi %u ooff %u nout %u tr0 %u\n", (int)blockIdx.x, rib, T,
           cnt, look, c_hi, ooff, nout, tr0);
    return;
  }
#endif
  if (DEFER && uni && nof == 32u && s <= 2u && (nlf == 2u || nlf == 3u)) {   // wave-uniform: every lane
    W->we = (int)nlf;
    W->A = (((C0f - 6u) >> 3) % (uint32_t)kRing) * kSlotBytes;
    W->ix = ix;
    W->acc = 0;
    W->b = ring[W->A + ix];                            // step 0's read
    W->ob = obf;
    // byte 0 of the window (its lowest address) relative to the shared base; other lanes
    // store out of range
    W->voff = walker ? (uint32_t)((uint64_t)(uintptr_t)(op - 31) - obf) : 0x80000000u;
    if (walker) nbytes = max(nbytes, ((chf - 14u) >> 3) + 1u);
    return;
  }
  if (!walker) return;
  if (uni) {
    uint32_t A = (((C0f - 6u) >> 3) % (uint32_t)kRing) * kSlotBytes;   // uniform slot base
    const uint32_t nl = (C0f - chf) >> 3;
    for (uint32_t i = 0; i < nl; i++) {                // lookahead blocks: state only
      ix = (ring[A + ix] & 63u) | rb;
      A = prevS(A);
    }
    for (uint32_t i = 0; i < nout; i++) {
      const uint32_t b = ring[A + ix];
      *op-- = (uint8_t)b;
      ix = (b & 63u) | rb;
      A = prevS(A);
    }
  } else {
    // previous slot: x - 1024, wrapping below slot 0 by one unsigned min (no compare + select)
    auto prev = [](uint32_t x) { const uint32_t y = x - (uint32_t)kSlotBytes; return min(y, y + span); };
    uint32_t a = (((C0 - 6u) >> 3) % (uint32_t)kRing) * kSlotBytes;
    for (uint32_t i = 0; i < nlook; i++) {
      ix = (ring[a + ix] & 63u) | rb;
      a = prev(a);
    }
    for (uint32_t i = 0; i < nout; i++) {
      const uint32_t b = ring[a + ix];
      *op-- = (uint8_t)b;
      ix = (b & 63u) | rb;
      a = prev(a);
    }
  }
  nbytes = max(nbytes, ((c_hi - 14u) >> 3) + 1u);
}

// P word of one column from its soft values (a, b) (BM(v, e) = e ? 14-2v : 2v, viterbilut.h):
// [BM(0,0), BM(0,1), BM(1,0), BM(1,1)] = (2a replicated ^ X) + ((2b replicated & Mb) ^ Y),
// with the lane's column kind in per-lane constants instead of selects (v_cndmask costs ~20
// cycles per wave on gfx950, profiles/r01_ubench_isa_costs.log):
// (halved: BM / 2 = e ? 7 - v : v = v ^ (e ? 7 : 0) for v = soft & 7)
//   full column (a on A, b on B): X = 0x07070000, Mb = ~0, Y = 0x07000700
//   A only:                        X = 0x07070000, Mb = 0,  Y = 0
//   B only (a on B):               X = 0x07000700, Mb = 0,  Y = 0
struct PKind {
  uint32_t X, Mb, Y;
};
__device__ __forceinline__ PKind p_kind(uint32_t r) {
  return r == 0 ? PKind{0x07070000u, 0xFFFFFFFFu, 0x07000700u}
                : (r == 1 ? PKind{0x07070000u, 0u, 0u} : PKind{0x07000700u, 0u, 0u});
}
// the same from bytes of an 8-byte pair {hi:lo}: selA / selB replicate byte a / b
__device__ __forceinline__ uint32_t p_word_sel(const PKind& k, uint32_t hi, uint32_t lo, uint32_t selA, uint32_t selB) {
  const uint32_t a1 = __builtin_amdgcn_perm(hi, lo, selA) & 0x07070707u;
  const uint32_t b1 = __builtin_amdgcn_perm(hi, lo, selB) & (0x07070707u & k.Mb);
  return (a1 ^ k.X) + (b1 ^ k.Y);
}
__device__ __forceinline__ uint32_t p_word(const PKind& k, uint32_t a, uint32_t b) {
  // v replicated into 4 bytes (v_perm), masked to v & 7 in each byte
  const uint32_t a1 = __builtin_amdgcn_perm(0u, a, 0u) & 0x07070707u;
  const uint32_t b1 = __builtin_amdgcn_perm(0u, b, 0u) & (0x07070707u & k.Mb);
  return (a1 ^ k.X) + (b1 ^ k.Y);
}

// DBG (timing experiments only, never selected by default): 1 skip the traceback walk,
// 2 skip snapshot stores, 4 skip normalization, 8 no P broadcast, 16 never run checked bodies,
// 64 ds_swizzle issued 4 columns ahead behind a scheduling barrier, 1024 no soft fetch
// (every body reuses the first body's soft values).  All are timing-only (wrong output).
constexpr int kPw = (24 + kLanes - 1) / kLanes;        // P words a lane builds per body (3 or 2)
// 8-lane rows: lane l builds the P words of body columns 3l .. 3l + 2, whose soft values are
// consecutive bytes, read as 2-3 dwords per body instead of 6 byte loads (ZRX_DWFETCH 0: the
// byte loads, lane l building columns l, 8 + l, 16 + l)
#ifndef ZRX_DWFETCH
#define ZRX_DWFETCH 1
#endif
constexpr bool kDwFetch = kLanes <= 8 && ZRX_DWFETCH != 0;
constexpr int kCpl = 24 / kLanes;                      // (kDwFetch) body columns a lane builds P words for
#ifndef ZRX_VPF
#define ZRX_VPF 1
#endif
constexpr int kPf = ZRX_VPF;                           // bodies the soft-value fetch runs ahead
// P words are broadcast kPq columns ahead of their column.  (Queues of 8 and 24, and each
// broadcast pinned where it is issued by a scheduling barrier, measured the same.)
constexpr int kPq = 4;
template <int CR, int DBG = 0>
struct Packet {
  using RT = Rate<CR>;
  const Consts& K;
  Row& R;
  uint32_t l, rib;
  uint8_t* ring;                                       // this body's first snapshot slot
  uint8_t* ring0;                                      // the block's ring (slot 0)
  Walk* W;                                             // deferred traceback tail (WS >= 0 bodies)
  RowX* rowx;                                          // the block's cold row facts (seam events)
  uint2* dumps;                                        // seam dumps

  // P word of body column J: lane J mod kLanes of the row built it as its word J / kLanes
  template <int J>
  static __device__ __forceinline__ uint32_t bcast(const uint32_t (&Pw)[kPw]) {
    if constexpr (kDwFetch)   // lane J / kCpl built columns kCpl l .. kCpl l + kCpl - 1
      return (uint32_t)__builtin_amdgcn_ds_swizzle((int)Pw[J % kCpl], ((J / kCpl) << 5) | (32 - kLanes));
    else
      return (uint32_t)__builtin_amdgcn_ds_swizzle((int)Pw[J / kLanes], ((J % kLanes) << 5) | (32 - kLanes));
  }
  // The deferred traceback steps of column J (branch-free; see Walk): steps 2J, 2J + 1 in
  // columns 0..11, step J + 12 after, NL + 32 steps in all.
  template <int J, int NL>
  __device__ __forceinline__ void walk_col() {
    constexpr bool fake = (DBG & 2048) != 0;
    if constexpr (J < 12) {
      walk_stepk<fake>(*W, (uint32_t)(2 * J), (uint32_t)NL, ring0, rib * 64u);
      walk_stepk<fake>(*W, (uint32_t)(2 * J + 1), (uint32_t)NL, ring0, rib * 64u);
    } else if constexpr (J + 12 < NL + 32) {
      walk_stepk<fake>(*W, (uint32_t)(J + 12), (uint32_t)NL, ring0, rib * 64u);
    }
  }
  // The half-1 snapshot bytes go out by asm without a memory clobber (one clobber per store
  // cost 0.7-1.5 %), so the compiler does not see them as LDS writes.  Invariant: no LDS read
  // of the ring may sit between a snapshot and the next compiler barrier — today the body's
  // end (`body`) and, in bodies with a deferred walk, the barrier after each snapshot (`col`).
  // events() and seam_event() read no ring slot (only rowx and global dumps); anything added
  // to a checked body that does must add a barrier.  -DZRX_SNAP_CLOBBER builds the stores with
  // the clobber: a parity A/B (scripts/build_flags_variant.sh) that shows a reordering as a
  // mismatch.
  template <uint32_t O>
static __device__ __forceinline__ void ds_b8_hi(uint32_t a, uint32_t v) {
#ifdef ZRX_SNAP_CLOBBER
  asm volatile("ds_write_b8_d16_hi %0, %1 offset:%2" ::"v"(a), "v"(v), "i"(O) : "memory");
#else
  asm volatile("ds_write_b8_d16_hi %0, %1 offset:%2" ::"v"(a), "v"(v), "i"(O));
#endif
}
// Snapshot k (column C = 8k + 6 of the body, C mod 6 = 2k): every position's pad byte
  // (bits 8..1 of its half) to the ring at the lane's first offset plus a lane-uniform delta.
  template <int k, int... D>
  __device__ __forceinline__ void snapshot(const uint32_t (&M)[kDw], std::integer_sequence<int, D...>) {
    uint8_t* s = ring + k * kSlotBytes;
    const uint32_t u[kDw] = {M[D]...};
    if constexpr (k == 2) {
      // C mod 6 = 4: position bits 0, 1 go to ring-index bits 1, 0, so (dword pair, half)
      // are 4 consecutive ring bytes, byte (h << 1) | (d & 1): one dword store per pair
      static_assert(snap_delta(2, 1, 0) == 1 && snap_delta(2, 0, 1) == 2, "k = 2 byte order");
#pragma unroll
      for (int e = 0; e < kDw / 2; e++)
        *(uint32_t*)(s + K.sa[2] + snap_delta(2, 2 * e, 0)) = __builtin_amdgcn_perm(u[2 * e + 1], u[2 * e], 0x06020400u);
    } else {
      // byte stores at constant offsets from one address: half 0 by a plain store (the
      // compiler emits and schedules ds_write_b8), half 1 by ds_write_b8_d16_hi (the
      // compiler would shift first).  The asm has no memory clobber (one per store cost
      // 0.7-1.5 %); the ordering that matters is kept by compiler barriers at the body's end
      // and, in bodies with a deferred walk, after each snapshot (col, body).
      uint8_t* b = s + K.sa[k];
      ((b[snap_delta(k, D, 0)] = (uint8_t)u[D]), ...);
      const uint32_t a = lds_addr(s) + K.sa[k];
      (ds_b8_hi<snap_delta(k, D, 1)>(a, u[D]), ...);
    }
  }
  template <int J, bool CHECKED, int WE, bool G, bool CHK>
  __device__ __forceinline__ void col(uint32_t (&M)[kDw], uint32_t (&Pq)[kPq], const uint32_t (&Pw)[kPw],
                                      uint32_t tr0, uint32_t& s_next, uint64_t dead, bool& ok) {
    if constexpr (WE > 0) walk_col<J, WE>();
    uint32_t P;
    if constexpr ((DBG & 8) != 0) {
      P = Pw[J / kLanes];
    } else {
      P = Pq[J % kPq];
      if constexpr (J + kPq < 24) Pq[J % kPq] = bcast<J + kPq>(Pw);   // issued kPq columns ahead
      if constexpr ((DBG & 64) != 0) __builtin_amdgcn_sched_barrier(0);
    }
    constexpr int r = J % RT::steps;
    constexpr int c = J + 1;                           // column index within the body after the step
    column5<J % 6, r, (J + 2) % 8, G>(M, P, K);
    if constexpr (CHK && (c == 6 || c == 12 || c == 18)) {   // guard-free body: some state has H <= 115
      // (one 16-bit compare into a lane mask: written as C++ it became an AND and a 32-bit compare)
      uint64_t lt;
      asm("v_cmp_gt_u16_e64 %0, %1, %2" : "=s"(lt) : "s"(0x3A00u), "v"(M[0]));   // (VOP3: no literal)
      const uint64_t pass = lt | dead;
      ok = ok & rows_all_any(pass);                    // (no short-circuit: a branch would split the body)
    }
    if constexpr (c % 8 == 6 && !(DBG & 2)) {
      snapshot<(c >> 3)>(M, std::make_integer_sequence<int, kDw>{});
      // A deferred walk (WE > 0) reads, in this body, slots that this body's snapshots then
      // overwrite: its loads must stay ahead of the half-1 asm stores, which the compiler
      // cannot see as memory writes
      if constexpr (WE > 0) asm volatile("" ::: "memory");
    }
    if constexpr (c % RT::steps == 0) {                // group end
      if constexpr (c % 8 == 0 && (CR != 2 || c == 24) && !(DBG & 4)) normalize(M);
      if constexpr (CHECKED) {
        const uint32_t tr = tr0 + c;
        if (tr >= s_next) {
          // seam events sit on body ends (seam columns are multiples of 24 from the row's start)
          // (a speculative body runs it only once its checks passed, so a redo never has to
          // restore the row's cold facts)
          if constexpr (c == 24)
            if (R.live && tr == R.evc && (!CHK || ok)) seam_event(R, tr, M, l, rib, rowx, dumps);
          events(R, tr, M);
          s_next = wave_min_rows(R.next);
        }
      }
    }
  }
  template <int... Q>
  static __device__ __forceinline__ void pq_fill(uint32_t (&Pq)[kPq], const uint32_t (&Pw)[kPw], std::integer_sequence<int, Q...>) {
    ((Pq[Q] = bcast<Q>(Pw)), ...);
  }
  // G: guard ANDs in every column; CHK: the guard-free body's H_min checks (returns whether
  // they all passed; rows in `dead` pass).  Rates 1/2 and 2/3 never need the guard.
  template <bool CHECKED, int WE, bool G, bool CHK, int... J>
  __device__ __forceinline__ bool body(uint32_t (&M)[kDw], const uint32_t (&Pw)[kPw], uint32_t tr0, uint32_t& s_next,
                                       std::integer_sequence<int, J...>, uint64_t dead = 0) {
    uint32_t Pq[kPq];
    bool ok = true;
    if constexpr (!(DBG & 8)) pq_fill(Pq, Pw, std::make_integer_sequence<int, kPq>{});
    (col<J, CHECKED, WE, G, CHK>(M, Pq, Pw, tr0, s_next, dead, ok), ...);
    // the tracebacks after a body read the slots its snapshots wrote (half 1 by asm stores
    // without a memory clobber): no load moves above this point
    asm volatile("" ::: "memory");
    return ok;
  }
};

// soft offset (within a body chunk) of body column j (constexpr form)
__host__ __device__ constexpr uint32_t soft_off_c(int cr, int j) {
  const int st = cr == 0 ? 1 : cr == 1 ? 2 : 3, G = cr == 0 ? 2 : cr == 1 ? 3 : 4;
  return (uint32_t)((j / st) * G + (j % st == 0 ? 0 : j % st + 1));
}
// soft offset (within a body chunk) and kind of body column j
template <int CR>
__device__ __forceinline__ uint32_t soft_off(uint32_t j) {
  constexpr uint32_t st = Rate<CR>::steps, G = Rate<CR>::G;
  const uint32_t g = j / st, r = j % st;
  return g * G + (r == 0 ? 0u : r + 1u);
}

// min / max of a row-uniform 64-bit value over the wave's rows (scalar)
__device__ __forceinline__ int64_t wave_min_rows64(int64_t v) {
  int64_t m = rl64(v, 0);
#pragma unroll
  for (int r = 1; r < kRowsWave; r++) m = min(m, rl64(v, r * kLanes));
  return m;
}
__device__ __forceinline__ int64_t wave_max_rows64(int64_t v) {
  int64_t m = rl64(v, 0);
#pragma unroll
  for (int r = 1; r < kRowsWave; r++) m = max(m, rl64(v, r * kLanes));
  return m;
}

// Issue priority of a SIMD's waves (run_rows).  ZRX_PRIO_MODE 1: the younger wave (odd block
// round) raises its priority in ZRX_PRIO_NUM of every ZRX_PRIO_DEN bodies.  2: the wave with
// the most columns left on its SIMD has it (g_vprog).  3: 2 for a mixed batch's planned rows,
// 1 otherwise.  0: off.  (Config 5, interleaved A/B with the ranked placement: 3 at 0.584-0.618
// ms, 1 at 0.597-0.629, within the boxes' spread; 2 on uniform batches: config 3 1.14-1.16 vs
// 1.13-1.14, config 2 0.41 vs 0.37 — the waves then run in lockstep and meet their
// traceback events together.  1 stays the default.)
#ifndef ZRX_PRIO_MODE
#define ZRX_PRIO_MODE 1
#endif
#ifndef ZRX_PRIO_NUM
#define ZRX_PRIO_NUM 2
#endif
#ifndef ZRX_PRIO_DEN
#define ZRX_PRIO_DEN 3
#endif
constexpr int kPrioMode = ZRX_PRIO_MODE, kPrioNum = ZRX_PRIO_NUM, kPrioDen = ZRX_PRIO_DEN;
// Columns left per resident wave: 16 words (HW_ID wave slots) per SIMD, the SIMD numbered
// from HW_ID / XCC_ID as (xcc, se, sh, cu, simd).  A wave writes its own word every body and
// 0 when it leaves; stale words of earlier launches are 0.  Only a speed hint: a wrong value
// changes which wave issues first, never what is computed.
constexpr int kProgSimds = 8 * 1024;
__device__ uint32_t g_vprog[kProgSimds * 16];
__device__ __forceinline__ uint32_t* prog_words(uint32_t& wid) {
  const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
  const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  wid = hw & 15u;
  const uint32_t s = (xcc & 7u) * 1024u + ((hw >> 13) & 7u) * 128u + ((hw >> 12) & 1u) * 64u + ((hw >> 8) & 15u) * 4u +
                     ((hw >> 4) & 3u);
  return g_vprog + 16u * s;
}
// max over the 16 lanes of each DPP row (every lane of the row gets it)
__device__ __forceinline__ uint32_t row16_max(uint32_t x) {
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xF, 0xF, false));   // row_ror:8
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x124, 0xF, 0xF, false));   // row_ror:4
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x122, 0xF, 0xF, false));   // row_ror:2
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x121, 0xF, 0xF, false));   // row_ror:1
  return x;
}
template <int CR, int DBG>
__device__ __forceinline__ void run_rows(const uint8_t* __restrict__ soft, int64_t so, uint32_t n, Row& R, const Consts& K, uint32_t l,
                         uint32_t rib, uint8_t* ring_block, uint8_t* __restrict__ out, uint32_t ooff,
                         uint32_t (&M)[kDw], RowX* rowx, uint2* __restrict__ dumps, bool prio, bool younger) {
  using RT = Rate<CR>;
  // guard ANDs outside the speculative bodies: rate 3/4 only (Guard-free columns)
  constexpr bool kG = CR == 2 || !kNoGuard;
  Walk W;
  W.we = 0;
  W.A = 0;
  W.ix = W.b = W.acc = 0;
  W.voff = 0x80000000u;
  W.ob = (uint64_t)(uintptr_t)out;
  Packet<CR, DBG> pk{K, R, l, rib, ring_block, ring_block, &W, rowx, dumps};
  // this lane builds the P words of body columns kLanes i + l (i < kPw; 16-lane rows: the
  // second word of lanes 8..15 repeats lanes 0..7's)
  // Soft values by buffer loads: one wave-uniform descriptor over the rows' soft windows,
  // advanced by the scalar unit every body, and a per-lane byte offset that never changes
  // (row offset + column offset).  Reads past the furthest row's last soft value fall outside
  // the descriptor and return 0; reads past a row's own end read its neighbour's values,
  // which feed only columns beyond R.cols.  The caller (k_viterbi3) passes rows whose soft
  // values lie within kSoftWindow of each other.
  const int64_t lo_me = R.live ? so : INT64_MAX, hi_me = R.live ? so + (int64_t)n : INT64_MIN;
  const int64_t lo_w = wave_min_rows64(lo_me) & ~(int64_t)3;   // (dword-aligned: soft is)
  const int64_t hi_w = (wave_max_rows64(hi_me) + 3) & ~(int64_t)3;
  if (hi_w - lo_w > kSoftWindow) {                     // one row's soft values beyond 4 GiB: not decodable
    if (R.live) R.nbytes = 0xFFFFFFFFu;
    return;
  }
  const uint32_t rel = R.live ? (uint32_t)(so - lo_w) : 0u;
  PKind kd[kPw];
  // kDwFetch: dwords dw0, +4, +8 hold this lane's bytes; word i's a / b are bytes sa_/sb_ of
  // {D1:D0} (or {D2:D1} for word 2 at rate 1/2)
  // 8 lanes: 2 dwords (3 at rate 1/2, word 2 from {D2:D1}); 4 lanes: word i from the pair
  // {D(k+1):Dk}, k = its first byte / 4 (the columns' byte offsets from column kCpl l repeat
  // every 6 columns, so k is a constant)
  constexpr int nD = !kDwFetch ? 2 * kPw : kLanes == 8 ? (CR == 0 ? 3 : 2) : (CR == 2 ? 3 : 4);
  uint32_t vo[kDwFetch ? 1 : kPw], selA[kPw], selB[kPw];
  if constexpr (kDwFetch) {
    const uint32_t j0 = (uint32_t)kCpl * l, off0 = soft_off<CR>(j0);
    const uint32_t w0 = rel + off0, sh = w0 & 3u;
    vo[0] = w0 & ~3u;
#pragma unroll
    for (int i = 0; i < kPw; i++) {
      kd[i] = p_kind((j0 + i) % RT::steps);
      uint32_t q = soft_off<CR>(j0 + i) - off0 + sh;
      if constexpr (kLanes == 8) {
        if (CR == 0 && i == 2) q -= 4u;                // from {D2:D1}
      } else {
        q -= 4u * (soft_off<CR>((uint32_t)i) >> 2);    // from the pair holding byte soft_off(i)
      }
      selA[i] = q * 0x01010101u;
      selB[i] = (q + 1u) * 0x01010101u;
    }
  } else {
#pragma unroll
    for (int i = 0; i < kPw; i++) {
      const uint32_t j = kLanes * i + ((kLanes * i + l < 24u) ? l : (l & 7u));
      vo[i] = soft_off<CR>(j) + rel;
      kd[i] = p_kind(j % RT::steps);
    }
  }
  // soft words / bytes of the next kPf bodies in flight (sd[0]: the next body's)
  uint32_t sd[kPf][nD];
  auto fetch_into = [&](uint32_t (&D)[nD], uint32_t base) {
    const int64_t left = hi_w - lo_w - (int64_t)base;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(soft + lo_w + base), (short)0, (int)(uint32_t)(left > 0 ? left : 0), 0x00020000);
    if constexpr (kDwFetch) {
#pragma unroll
      for (int d = 0; d < nD; d++) D[d] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)vo[0] + 4 * d, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < kPw; i++) {
        D[2 * i] = __builtin_amdgcn_raw_buffer_load_b8(rs, (int)vo[i], 0, 0);
        D[2 * i + 1] = __builtin_amdgcn_raw_buffer_load_b8(rs, (int)vo[i] + 1, 0, 0);
      }
    }
  };
  // P words of the body at `base` from sd[0], then the fetch window moves one body on
  auto pwords = [&](uint32_t (&Pw)[kPw], uint32_t base_) {
#pragma unroll
    for (int i = 0; i < kPw; i++) {
      if constexpr (kDwFetch) {
        const int k = kLanes == 8 ? ((CR == 0 && i == 2) ? 1 : 0) : (int)(soft_off_c(CR, i) >> 2);
        Pw[i] = p_word_sel(kd[i], sd[0][k + 1], sd[0][k], selA[i], selB[i]);
      } else {
        Pw[i] = p_word(kd[i], sd[0][2 * i], sd[0][2 * i + 1]);
      }
    }
    if constexpr ((DBG & 1024) == 0) {
#pragma unroll
      for (int q = 0; q + 1 < kPf; q++)
#pragma unroll
        for (int i = 0; i < nD; i++) sd[q][i] = sd[q + 1][i];
      fetch_into(sd[kPf - 1], base_ + kPf * RT::chunk);   // (latency hidden behind kPf bodies)
    }
  };
#pragma unroll
  for (int q = 0; q < kPf; q++) fetch_into(sd[q], q * RT::chunk);
  uint32_t s_next = wave_min_rows(R.next);
  uint32_t slot = 0;                                   // first slot of this body (3 per body)
  uint32_t tr0 = 0, base = 0;
  constexpr auto cols24 = std::make_integer_sequence<int, 24>{};
  // Issue priority: a SIMD's two waves come from blocks b and b + ncu, and with equal
  // priority the SIMD always issues the older one first, so it runs at nearly full speed and
  // the younger one finishes alone long after it (and in a mixed batch a long wave beside a
  // short one runs at the shared speed, then alone).  Mode 2: every body, the wave with more
  // columns left than any other wave on its SIMD (their words loaded one body earlier) takes
  // priority 1 — longest remaining first, so the SIMD's waves end together and a long wave
  // beside short ones runs at nearly its lone speed.  Mode 1: the younger wave raises its
  // priority in NUM of every DEN bodies.
  uint32_t pc = 0;
  uint32_t wid = 0, pv = 0;
  uint32_t* const pw = kPrioMode >= 2 && prio ? prog_words(wid) : g_vprog;
  // the SIMD's 16 words by buffer ops with sc0: read from this XCD's L2, where the other
  // waves of this CU write them (agent-scope atomics go past the L2 to memory: 1.51 ms
  // instead of 1.14, whole CUs slowed by the round trips)
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc((void*)pw, (short)0, 64, 0x00020000);
  constexpr int kSc0 = 1;
  const uint32_t wend = kPrioMode >= 2 && prio ? (uint32_t)wave_max_rows64(R.live ? (int64_t)R.cols : 0) : 0u;
  const uint32_t lane = __lane_id();
  auto next_body = [&]() {
    slot = slot + 3 == kRing ? 0 : slot + 3;
    tr0 += 24;
    base += RT::chunk;
    if constexpr (kPrioMode >= 2) {
      if (prio) {
        const uint32_t rem = wend > tr0 ? wend - tr0 : 0u;
        const uint32_t om = (uint32_t)__builtin_amdgcn_readfirstlane((int)row16_max(lane < 16u && lane != wid ? pv : 0u));
        if (rem > om) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
    }
    if constexpr (kPrioMode != 2 && kPrioNum > 0) {
      if (younger) {
        pc = pc + 1 == (uint32_t)kPrioDen ? 0u : pc + 1;
        if (pc < (uint32_t)kPrioNum) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
    }
  };
  // Mode 2's own word and the SIMD's words, at the start of a body (before its soft prefetch,
  // so next_body's wait for pv leaves the prefetch in flight): the store and load then have
  // the whole body to complete.
  // (Every lane stores / loads: a lane-masked memory op is a branch, and the waitcnt pass then
  // drains everything in flight at the loop head; issued at the body's end, the loop head's
  // wait for the prefetch also waited for them: 1.63 ms instead of 1.14.)
  auto publish = [&]() {
    if constexpr (kPrioMode >= 2) {
      if (prio) {
        __builtin_amdgcn_raw_buffer_store_b32(wend > tr0 ? wend - tr0 : 0u, prs, (int)(4u * wid), 0, kSc0);
        pv = __builtin_amdgcn_raw_buffer_load_b32(prs, (int)(4u * (lane & 15u)), 0, kSc0);
      }
    }
  };
  while (__builtin_amdgcn_ballot_w64(R.live) != 0) {
    // The hot loop: bodies with no event due, no deferred walk, nothing else on this path
    // (its own loop, so the register allocator keeps the loop-carried values in place).
    while ((DBG & 16) || (s_next > tr0 + 24 && s_next != kNever)) {
      uint32_t Pw[kPw];
      publish();
      pwords(Pw, base);
      pk.ring = ring_block + slot * kSlotBytes;
      if constexpr (CR == 2 && kNoGuard) {             // speculative guard-free body, redone on a failed check
        uint32_t M0[kDw];
#pragma unroll
        for (int d = 0; d < kDw; d++) M0[d] = M[d];
        const uint64_t dead = __builtin_amdgcn_ballot_w64(!R.live);
        if (!pk.template body<false, 0, false, true>(M, Pw, tr0, s_next, cols24, dead)) {
#pragma unroll
          for (int d = 0; d < kDw; d++) M[d] = M0[d];
          pk.template body<false, 0, true, false>(M, Pw, tr0, s_next, cols24);
        }
      } else {
        pk.template body<false, 0, kG, false>(M, Pw, tr0, s_next, cols24);
      }
      next_body();
      if constexpr ((DBG & 16) != 0) {                 // no events: stop at the input's end
        if (tr0 >= R.cols) R.live = false;
        if (__builtin_amdgcn_ballot_w64(R.live) == 0) break;
      }
    }
    if constexpr ((DBG & 16) != 0) break;
    if (s_next == kNever) break;                       // every row is done
    // A body with an event due: checked, then the tracebacks it raised.
    {
      uint32_t Pw[kPw];
      publish();
      pwords(Pw, base);
      pk.ring = ring_block + slot * kSlotBytes;
      if constexpr (CR == 2 && kNoGuard) {             // speculative too: events restored with the metrics
        uint32_t M0[kDw];
#pragma unroll
        for (int d = 0; d < kDw; d++) M0[d] = M[d];
        const Row R0 = R;
        const uint32_t s0 = s_next;
        if (!pk.template body<true, 0, false, true>(M, Pw, tr0, s_next, cols24, __builtin_amdgcn_ballot_w64(!R.live))) {
#pragma unroll
          for (int d = 0; d < kDw; d++) M[d] = M0[d];
          R = R0;
          s_next = s0;
          pk.template body<true, 0, true, false>(M, Pw, tr0, s_next, cols24);
        }
      } else {
        pk.template body<true, 0, kG, false>(M, Pw, tr0, s_next, cols24);
      }
    }
    if ((DBG & 1) == 0 && __builtin_amdgcn_ballot_w64(R.ppend) != 0) {
      traceback<true>(R.ppend, R.pM, R.pT, 256u, R.plook, l, rib, ring_block, out, ooff, R.nbytes, &W, tr0);
      walk_uniform(W);
      R.ppend = false;
    }
    if ((DBG & 1) == 0 && __builtin_amdgcn_ballot_w64(R.fpend) != 0) {
      traceback(R.fpend, R.fM, R.fT, R.fcnt, R.flook, l, rib, ring_block, out, ooff, R.nbytes);
      R.fpend = false;
    }
    if constexpr ((DBG & 1) != 0) R.ppend = R.fpend = false;
    next_body();
    // A deferred traceback walk runs in the next body's columns.
    if (W.we && __builtin_amdgcn_ballot_w64(R.live) != 0) {
      uint32_t Pw[kPw];
      publish();
      pwords(Pw, base);
      pk.ring = ring_block + slot * kSlotBytes;
      // No event due in this body (the usual case: a wave's windows end together, one body
      // before): the walk rides an unchecked body, and only the metrics need a copy.
      const bool quiet = s_next > tr0 + 24 && s_next != kNever;
      if constexpr (CR == 2 && kNoGuard) {
        // speculative: on a failed check the body is redone without the walk, whose reads all
        // came before this body's snapshot stores and from verified bodies' slots (Walk), so
        // its bytes already stored are right
        uint32_t M0[kDw];
#pragma unroll
        for (int d = 0; d < kDw; d++) M0[d] = M[d];
        if (quiet) {
          const uint64_t dead = __builtin_amdgcn_ballot_w64(!R.live);
          const bool ok = W.we == 3 ? pk.template body<false, 3, false, true>(M, Pw, tr0, s_next, cols24, dead)
                                    : pk.template body<false, 2, false, true>(M, Pw, tr0, s_next, cols24, dead);
          if (!ok) {
#pragma unroll
            for (int d = 0; d < kDw; d++) M[d] = M0[d];
            pk.template body<false, 0, true, false>(M, Pw, tr0, s_next, cols24);
          }
        } else {
          const Row R0 = R;
          const uint32_t s0 = s_next;
          const uint64_t dead = __builtin_amdgcn_ballot_w64(!R.live);
          const bool ok = W.we == 3 ? pk.template body<true, 3, false, true>(M, Pw, tr0, s_next, cols24, dead)
                                    : pk.template body<true, 2, false, true>(M, Pw, tr0, s_next, cols24, dead);
          if (!ok) {
#pragma unroll
            for (int d = 0; d < kDw; d++) M[d] = M0[d];
            R = R0;
            s_next = s0;
            pk.template body<true, 0, true, false>(M, Pw, tr0, s_next, cols24);
          }
        }
      } else if (quiet) {
        if (W.we == 3) pk.template body<false, 3, kG, false>(M, Pw, tr0, s_next, cols24);
        else pk.template body<false, 2, kG, false>(M, Pw, tr0, s_next, cols24);
      } else {
        if (W.we == 3) pk.template body<true, 3, kG, false>(M, Pw, tr0, s_next, cols24);
        else pk.template body<true, 2, kG, false>(M, Pw, tr0, s_next, cols24);
      }
      W.we = 0;
      if ((DBG & 1) == 0 && __builtin_amdgcn_ballot_w64(R.fpend) != 0) {   // (a partial window is 256 columns on)
        traceback(R.fpend, R.fM, R.fT, R.fcnt, R.flook, l, rib, ring_block, out, ooff, R.nbytes);
        R.fpend = false;
      }
      if constexpr ((DBG & 1) != 0) R.ppend = R.fpend = false;
      next_body();
    }
  }
  if constexpr (kPrioMode >= 2) {
    if (prio) {                                        // leaving: no columns left
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_raw_buffer_store_b32(0u, prs, (int)(4u * wid), 0, kSc0);
    }
  }
  if (W.we) walk_finish(W, ring_block, rib * 64u);     // rows done before the deferred tail ran
}

}  // namespace v3

// vparams[4p..] = {frame_len, code_rate, soft_len, *}; out_bits[p] = bits written.
// Requires depth 256 (the only depth the WiFi RX uses: Viterbi.blk:34).  Four rows per wave
// (16 lanes each); rows of a wave may have different rates and lengths (a wave runs one pass
// per rate present), so batches are first planned by k_pkt_plan.
//   rows:  the plan's row table, {packet, k | nseg << 8} per slot, *nrows_p of them (a row is
//          segment k of nseg of its packet); null: slot = packet, whole frames (nslots).
//   fix:   the seam pass after a planned launch: slot = packet (segs[p] = its nseg); a row
//          re-decodes from the first seam whose two dumps disagree (usually none).
// The grid may be smaller than the rows (block-stride loop).
#ifdef ZRX_VTRACE
// (timeline probe builds only: scripts/exp/vit_trace.py, in git history at e0a0913) 8 words per row slot: start and end
// (s_memrealtime, 100 MHz, low words), HW_ID, XCC_ID, block, columns, rate, packet
__device__ uint32_t* g_vtrace;
__device__ uint32_t g_vtrace_rows;                     // row slots the buffer holds
#endif
template <int DBG, bool FIX>
__device__ __forceinline__ void viterbi_rows(int g0, int nrows, uint32_t uni, uint32_t ncu, uint32_t ncu_rcp,
                                             const v3::Consts& K, uint8_t* ring, v3::RowX* rowx,
                                             const uint8_t* __restrict__ soft, const int64_t* __restrict__ soft_off,
                                             const int32_t* __restrict__ vparams, uint8_t* __restrict__ out,
                                             const int64_t* __restrict__ out_off, int32_t* __restrict__ out_bits,
                                             const int2* __restrict__ rows, const uint8_t* __restrict__ segs,
                                             uint2* __restrict__ dumps, int32_t* __restrict__ stats) {
  constexpr int fix = FIX;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t l = lane & (v3::kLanes - 1u);
  const uint32_t rib = threadIdx.x >> v3::kLaneBits;   // row in block
#ifdef ZRX_VTRACE
  const uint32_t vt0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
  {
    const int slot = g0 + (int)rib;
    bool valid = slot < nrows;
    int p = slot;
    uint32_t k = 0, nseg = 1;
    if (valid && rows) {
      if (uni) {
        // a uniform batch: row r = segment r / np of packet r mod np (np = nrows / u), so a
        // wave's rows are one segment index of consecutive packets: their windows line up
        // (the deferred walk is per wave) whatever the warm-up
        const uint32_t r = v3::order_place((uint32_t)slot, (uint32_t)nrows / v3::kRows, ncu, ncu_rcp);
        const uint32_t np = (uint32_t)nrows / uni;
        k = r / np; p = (int)(r - k * np); nseg = uni;
      } else {
        const int2 r = rows[slot];
        p = r.x; k = (uint32_t)r.y & 0xFFu; nseg = ((uint32_t)r.y >> 8) & 0xFFu;
        if (p < 0) { valid = false; p = 0; nseg = 1; k = 0; }   // a slot the wave placement left empty
      }
    }
#ifdef ZRX_GUARD
    if (valid && ((uint32_t)p >= v3::g_zg_np || nseg == 0 || nseg > (uint32_t)v3::kMaxSeg || k >= nseg)) {
      printf("ZG row bad: blk %d rib %u slot %d p %d k %u nseg %u fix %d\n", (int)blockIdx.x, rib, slot, p, k, nseg, fix);
      return;
    }
#endif
    if (valid && fix) nseg = uni ? uni : segs[p];
#ifdef ZRX_GUARD
    if (valid && fix && nseg > (uint32_t)v3::kMaxSeg) {
      printf("ZG segs bad: p %d nseg %u\n", p, nseg);
      nseg = 1;
    }
#endif
    const bool load = valid && (!fix || nseg > 1u);
    int fl = 0, cr = 0, n = 0;
    int64_t so = 0, oo = 0;
    if (load) {
      const int32_t* vp = vparams + 4 * (int64_t)p;
      fl = vp[0]; cr = vp[1]; n = vp[2];
      so = soft_off[p]; oo = out_off[p];
    }
    const uint32_t W = uni ? v3::kSegWarmUni : v3::kSegWarm;   // warm-up of the segments
    const uint32_t cols = load && n > 0 && cr >= 0 && cr <= 2 ? (uint32_t)(n / (cr == 0 ? 2 : cr == 1 ? 3 : 4)) * (uint32_t)(cr + 1) : 0u;
    const uint32_t E = (uint32_t)fl * 8u + 6u;
    // this row's segment: first column S, last column, seam j of its first seam event
    uint32_t S = 0, stop = cols, j = 0;
    bool work = cols > 0;
    if constexpr (FIX) {
      // The first (ks) and last (kl) seams whose sides disagree: the fix row starts at ks
      // from segment ks - 1's state and may stop only at a later seam past kl whose start
      // state it reproduces (every segment after that one then starts right).
      uint32_t ks = 0, kl = 0;
      for (uint32_t jj = 1; __builtin_amdgcn_ballot_w64(work && jj < nseg) != 0; jj++) {
        const bool ne = work && jj < nseg &&
                        v3::dump_ne(dumps + v3::seam_index((uint32_t)p, jj, 0), dumps + v3::seam_index((uint32_t)p, jj, 1), l);
        const uint64_t bad = __builtin_amdgcn_ballot_w64(ne);
        if (v3::row_bits(bad) != 0u) {
          if (ks == 0u) ks = jj;
          kl = jj;
        }
      }
      work = work && ks != 0u;
      if (work) { S = v3::seg_start(E, nseg, ks, W) + v3::seg_cmp(W); j = kl + 1u; k = ks; }
#ifdef ZRX_GUARD
      if (work && l == 0)
        printf("ZG fix row: blk %d rib %u p %d nseg %u ks %u S %u E %u cols %u cr %d n %d\n", (int)blockIdx.x, rib, p, nseg,
               ks, S, E, cols, cr, n);
#endif
      if (work && l == 0 && stats) atomicAdd(stats + 1, 1);
    } else if (nseg > 1u && work) {
      S = v3::seg_start(E, nseg, k, W);
      stop = v3::seg_stop(E, cols, nseg, k, W);
      j = k ? k : 1u;
    }
    // (cold facts in LDS: read back where needed instead of held in registers by the decode)
    // (fix rows: k holds ks, the seam they start at)
    rowx[rib] = v3::RowX{(uint32_t)p, k | (nseg << 8) | ((uint32_t)(fix != 0) << 16) | ((uint32_t)(uni != 0u) << 18) | (j << 20),
                         S, E};
    const int64_t sS = work ? (int64_t)(S / (uint32_t)(cr + 1)) * (cr == 0 ? 2 : cr == 1 ? 3 : 4) : 0;   // soft values before S
    so += sS;
    const uint32_t nS = work ? (uint32_t)((int64_t)n - sS) : 0u;
    const uint32_t colsS = work ? min(cols, stop) - S : 0u;
    oo += S >> 3;
    // output bytes are addressed as out + 32-bit offset (one uniform base for the whole wave)
    uint8_t* obase = out + (oo & ~(int64_t)0xFFFFFFFF);
    const uint32_t ooff = (uint32_t)(oo & 0xFFFFFFFF);
    uint32_t nbytes = 0;
    // rows of one rate run together; other rows of the wave sit out that pass.  The row state
    // is built per pass (not kept across passes), which keeps it out of the register budget.
    for (int rate = 0; rate < 3; rate++) {
      const bool mine = work && cr == rate;
      if (__builtin_amdgcn_ballot_w64(mine) == 0) continue;
      // The soft values of a pass's rows are read through one 32-bit buffer window (run_rows);
      // rows further apart than that run one at a time (correct, 4x the time; only batches
      // with more than 4 GiB of soft values can get there).
      const int64_t lo_me = mine ? so : INT64_MAX, hi_me = mine ? so + (int64_t)nS : INT64_MIN;
      const int64_t lo_w = v3::wave_min_rows64(lo_me);
      const int64_t hi_w = v3::wave_max_rows64(hi_me);
      const int passes = hi_w - lo_w > v3::kSoftWindow ? v3::kRowsWave : 1;
      for (int q = 0; q < passes; q++) {
        const bool mq = mine && (passes == 1 || (int)(rib % v3::kRowsWave) == q);
        if (__builtin_amdgcn_ballot_w64(mq) == 0) continue;
        // start state, output base and first seam event of the row (v3::seg_start)
        const v3::RowX x = rowx[rib];
        const uint32_t xk = x.kn & 0xFFu, xn = (x.kn >> 8) & 0xFFu, xj = x.kn >> 20;
        const bool xfix = (x.kn >> 16) & 1u;
        const uint32_t xw = (x.kn >> 18) & 1u ? v3::kSegWarmUni : v3::kSegWarm;
        uint32_t M[v3::kDw];
        if (xfix && mq) {                               // segment ks - 1's exact state at S = C_ks
          v3::dump_load(dumps + v3::seam_index(x.p, x.kn & 0xFFu, 0), l, M);
        } else if (xk) {                                // warm-up from zero
#pragma unroll
          for (int d = 0; d < v3::kDw; d++) M[d] = 0u;
        } else {                                        // ALL_INIT0 (viterbilut.h:74-82)
#pragma unroll
          for (int d = 0; d < v3::kDw; d++)
            M[d] = ((v3::pos_of(l, d, 1) ? 24u : 0u) << 24) | ((v3::pos_of(l, d, 0) ? 24u : 0u) << 8);   // 48 >> 1
        }
        // issue priority (run_rows): longest remaining first for a mixed batch's rows, the
        // younger wave's 2 of 3 bodies otherwise
        const bool mixed = rows != nullptr && uni == 0u;
        const bool lrpt = !FIX && (v3::kPrioMode == 2 || (v3::kPrioMode == 3 && mixed));
        const bool younger = !FIX && (v3::kPrioMode == 1 || (v3::kPrioMode == 3 && !mixed)) && ((blockIdx.x / ncu) & 1u) != 0u;
#if defined(ZRX_STAGGER) && ZRX_STAGGER > 0
        if (younger) __builtin_amdgcn_s_sleep(ZRX_STAGGER);   // (experiment: offset the SIMD's two waves)
#endif
        v3::Row Rr;
        Rr.ob = xfix ? xw - v3::seg_cmp(xw) : xk ? xw : 0u;
        Rr.end = x.E - x.S; Rr.cols = colsS;
        Rr.evc = xj != 0u && xj < xn ? v3::seg_start(x.E, xn, xj, xw) + v3::seg_cmp(xw) - x.S : v3::kNever;
        Rr.live = mq;
        Rr.ppend = Rr.fpend = false;
        Rr.pT = Rr.plook = Rr.fT = Rr.fcnt = Rr.flook = 0;
#pragma unroll
        for (int d = 0; d < v3::kDw; d++) Rr.pM[d] = Rr.fM[d] = 0u;
        Rr.nbytes = 0;
        Rr.next = v3::row_next(Rr);
        if (rate == 0) v3::run_rows<0, DBG>(soft, so, nS, Rr, K, l, rib, ring, obase, ooff, M, rowx, dumps, lrpt, younger);
        else if (rate == 1) v3::run_rows<1, DBG>(soft, so, nS, Rr, K, l, rib, ring, obase, ooff, M, rowx, dumps, lrpt, younger);
        else v3::run_rows<2, DBG>(soft, so, nS, Rr, K, l, rib, ring, obase, ooff, M, rowx, dumps, lrpt, younger);
        if (mq) nbytes = Rr.nbytes;
      }
    }
    // the frame's bit count: from its last segment, or from a fix row that ran to the end
    if (valid && l == 0) {
      const v3::RowX x = rowx[rib];
      const uint32_t xk = x.kn & 0xFFu, xn = (x.kn >> 8) & 0xFFu;
      const bool last = (x.kn >> 16) & 1u ? work && ((x.kn >> 17) & 1u) == 0u : xk + 1u == xn;
      if (last) out_bits[x.p] = nbytes == 0xFFFFFFFFu ? -1 : (int32_t)((nbytes + (x.S >> 3)) * 8u);
    }
#ifdef ZRX_VTRACE
    if (!FIX && valid && l == 0 && g_vtrace && (uint32_t)slot < g_vtrace_rows) {
      uint32_t* r = g_vtrace + 8 * (size_t)slot;
      r[0] = vt0;
      r[1] = (uint32_t)__builtin_amdgcn_s_memrealtime();
      r[2] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
      r[3] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);
      r[4] = blockIdx.x; r[5] = colsS; r[6] = (uint32_t)cr; r[7] = (uint32_t)p;
    }
#endif
  }
}
template <int DBG, bool FIX = false>
__global__ __launch_bounds__(256, v3::kWavesPerSimd) void k_viterbi3(const uint8_t* __restrict__ soft, const int64_t* __restrict__ soft_off,
                                                  const int32_t* __restrict__ vparams, int nslots,
                                                  uint8_t* __restrict__ out, const int64_t* __restrict__ out_off,
                                                  int32_t* __restrict__ out_bits, const int2* __restrict__ rows,
                                                  int32_t* __restrict__ nrows_p, const uint8_t* __restrict__ segs,
                                                  uint2* __restrict__ dumps) {
  __shared__ uint8_t ring[v3::kRing * v3::kSlotBytes];
  __shared__ v3::RowX rowx[v3::kRows];
  // the plan header (v3::PlanWord): rows, the fix pass's count of re-decoded rows, the
  // segments per packet of a uniform batch (0: row table), the CU count of the placement
  const int nrows = FIX || !nrows_p ? nslots : nrows_p[v3::kPlanRows];
  const uint32_t uni = nrows_p ? (uint32_t)nrows_p[v3::kPlanUniform] : 0u;
  const uint32_t ncu = nrows_p ? max((uint32_t)nrows_p[v3::kPlanNcu], 2u) : 2u;
  const uint32_t ncu_rcp = 0xFFFFFFFFu / ncu + 1u;
  if (FIX && uni == 1u) return;                        // a uniform batch of whole frames has no seams
  v3::Consts K;
  v3::make_consts(K, threadIdx.x & (v3::kLanes - 1u), threadIdx.x >> v3::kLaneBits);
  if constexpr (FIX) {                                 // block-stride over the packets
    for (int g0 = blockIdx.x * v3::kRows; g0 < nrows; g0 += gridDim.x * v3::kRows)
      viterbi_rows<DBG, true>(g0, nrows, uni, ncu, ncu_rcp, K, ring, rowx, soft, soft_off, vparams, out, out_off, out_bits, rows, segs, dumps,
                              nrows_p);
  } else {
    const int g0 = blockIdx.x * v3::kRows;
    if (g0 < nrows)
      viterbi_rows<DBG, false>(g0, nrows, uni, ncu, ncu_rcp, K, ring, rowx, soft, soft_off, vparams, out, out_off, out_bits, rows, segs,
                               dumps, nullptr);
  }
}

// Row order for k_viterbi3 (k_pkt_plan): by code rate, then by trellis length of the row
// (a frame or one of its segments), longest first, so the four rows of a wave share one rate
// and similar lengths.  Counting sort over (rate, 24-column bodies) keys; 1024 length buckets
// cover 24576 columns, i.e. every 802.11a frame (at most 8 x 2050 + 6 = 16406 columns);
// longer device-API frames share the last bucket.  Within a bucket the order is whatever the
// atomics give (each row decodes the same wherever it lands).
constexpr int kOrderLen = 1024;                        // length buckets of 24 columns
constexpr int kOrderKeys = 3 * kOrderLen + 1;          // + one bucket for packets with no work
constexpr int kOrderPerThread = (kOrderKeys + 1023) / 1024;
__device__ __forceinline__ uint32_t order_key_len(int cr, uint32_t len) {
  if (len == 0 || cr < 0 || cr > 2) return 3u * kOrderLen;
  const uint32_t bodies = min((len + 23u) / 24u, (uint32_t)kOrderLen - 1u);
  return (uint32_t)cr * kOrderLen + (kOrderLen - 1u - bodies);
}
// trellis columns of a packet's soft input (constant divisors)
__device__ __forceinline__ uint32_t cols_of(int cr, int n) {
  if (n <= 0 || cr < 0 || cr > 2) return 0u;
  const uint32_t u = (uint32_t)n;
  return cr == 0 ? u >> 1 : cr == 1 ? (u / 3u) * 2u : (u >> 2) * 3u;
}
// Adds this wave's valid lanes to hist[key] and returns each lane's slot (old count + rank
// among the lanes sharing its key).  The lanes of the wave's first two keys are counted with
// one atomic each (a uniform batch has one key, the segments of a mixed one few), the rest
// one atomic per lane, so lanes sharing a key do not serialize on one LDS address.
__device__ __forceinline__ uint32_t order_claim(uint32_t* hist, bool valid, uint32_t key) {
  uint64_t rem = __builtin_amdgcn_ballot_w64(valid);
  uint32_t slot = 0;
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (int it = 0; it < 2; it++) {
    if (rem == 0) return slot;
    const uint32_t first = (uint32_t)__builtin_ctzll(rem);
    const uint32_t k0 = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)first);
    const uint64_t m = __builtin_amdgcn_ballot_w64(valid && key == k0);
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(&hist[k0], (uint32_t)__builtin_popcountll(m));
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)first);
    if ((m >> lane) & 1u) slot = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    rem &= ~m;
  }
  if ((rem >> lane) & 1u) slot = atomicAdd(&hist[key], 1u);
  return slot;
}
// hist[] counts -> exclusive starts (1024 threads, kOrderPerThread buckets each); returns the
// total.  The caller syncs before and after.
__device__ __forceinline__ uint32_t order_hist_scan(uint32_t* hist) {
  __shared__ uint32_t wsum[16];
  const int t = threadIdx.x;
  uint32_t v[kOrderPerThread], mine = 0;
#pragma unroll
  for (int j = 0; j < kOrderPerThread; j++) { v[j] = hist[kOrderPerThread * t + j]; mine += v[j]; }
  uint32_t inc = mine;                                 // inclusive scan inside the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = (uint32_t)__shfl_up((int)inc, o);
    if ((t & 63) >= o) inc += u;
  }
  if ((t & 63) == 63) wsum[t >> 6] = inc;
  __syncthreads();
  uint32_t ex = inc - mine, total = 0;
  for (int w = 0; w < (t >> 6); w++) ex += wsum[w];
  for (int w = 0; w < 16; w++) total += wsum[w];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kOrderPerThread; j++) { hist[kOrderPerThread * t + j] = ex; ex += v[j]; }
  return total;
}

}  // namespace zrx




