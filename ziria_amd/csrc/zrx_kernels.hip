// MI355X (gfx950) kernels of the 802.11a RX decode hot path.
//
//   k_fft64          one 64-point FFT per lane (FFT<64>, csrc/fft_r4difx.hpp:220-237)
//   k_signal_fft     SIGNAL symbol per lane: FFT -> GetData -> DemapLimit -> DemapBPSK ->
//                    DeinterleaveBPSK (DecodePLCP.blk:30-37)
//   k_signal_vit     one row per packet (v3 layout): Viterbi_sig11 (viterbicore.hpp:272-315) +
//                    parsePLCPHeader (parsePLCPHeader.blk:119-213)
//   k_data_fft       lane = data symbol, flat over the batch: FFT -> GetData -> DemapLimit ->
//                    Demap{mod} -> Deinterleave{mod} (Decode.blk:45-60); with EQ, ChannelEqualization
//                    + PilotTrack after the FFT (receiver.blk:66-71), also in k_signal_fft
//   k_ofdm_eq        FFT -> ChannelEqualization -> PilotTrack, full 64-bin output
//   k_viterbi3       (zrx_viterbi3.hpp) the batched brick driver loop, four packets per wave
//   k_descramble_crc one wave per packet: descrambler (Decode.blk:36-43) + CRC-32 check
//                    (crc.blk:85-118), 64 lanes each on a chunk, CRC combined by GF(2) maps
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zrx_device.hpp"
#include "zrx_viterbi3.hpp"
#include "zrx_frontend.hpp"
#include "zrx_tx.hpp"
#include "zrx_fftn.hpp"

namespace zrx {

constexpr int kDecStride = 2080;      // decoded bytes per packet in the rx chain (len+2 <= 2050)
constexpr int kPayloadStride = 4096;  // payload bytes per packet

// ------------------------------------------------------------------ FFT64 batch
__global__ __launch_bounds__(256) void k_fft64(const uint4* __restrict__ in, uint4* __restrict__ out,
                                               int64_t nsym) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsym) return;
  s2 x[64];
  const uint4* src = in + s * 16;
#pragma unroll
  for (int q = 0; q < 16; q++) {
    const uint4 v = src[q];
    x[4 * q] = as_s2(v.x); x[4 * q + 1] = as_s2(v.y); x[4 * q + 2] = as_s2(v.z); x[4 * q + 3] = as_s2(v.w);
  }
  fft64_inplace(x);
  uint4* dst = out + s * 16;
#pragma unroll
  for (int q = 0; q < 16; q++) {
    dst[q] = make_uint4(as_u32(x[bitrev6(4 * q)]), as_u32(x[bitrev6(4 * q + 1)]),
                        as_u32(x[bitrev6(4 * q + 2)]), as_u32(x[bitrev6(4 * q + 3)]));
  }
}

__device__ __forceinline__ void load_symbol(const uint4* __restrict__ src, s2* x) {
#pragma unroll
  for (int q = 0; q < 16; q++) {
    const uint4 v = src[q];
    x[4 * q] = as_s2(v.x); x[4 * q + 1] = as_s2(v.y); x[4 * q + 2] = as_s2(v.z); x[4 * q + 3] = as_s2(v.w);
  }
}

// (blocks of a multiple of 64 threads: every load issued before the first store, one memory
// latency; a strided loop over blockDim waited for each of its rounds in turn)
__device__ __forceinline__ void stage_lut(uint32_t* lut) {
  const uint32_t t = threadIdx.x & 63u;
  uint32_t v[4];
#pragma unroll
  for (int k = 0; k < 4; k++) v[k] = kDemapLut[t + 64 * k];
#pragma unroll
  for (int k = 0; k < 4; k++) lut[t + 64 * k] = v[k];
  __syncthreads();
}

// ------------------------------------------------------------------ SIGNAL symbol -> 48 soft
// EQ: ChannelEqualization (coefficients chan[64p ..]) + PilotTrack between FFT and GetData
// (receiver.blk:66-71); otherwise the FFT output feeds GetData directly.
template <bool EQ>
__global__ __launch_bounds__(256) void k_signal_fft(const uint4* __restrict__ sym, const int64_t* __restrict__ sym_off,
                                                    const int32_t* __restrict__ nsym, int npkts,
                                                    uint4* __restrict__ sig_soft, const uint32_t* __restrict__ chan,
                                                    EqTabs T) {
  __shared__ uint32_t lut[256];
  stage_lut(lut);
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npkts) return;
  uint32_t w[12];
  if (nsym[p] >= 1) {
    s2 x[64];
    load_symbol(sym + sym_off[p] * 16, x);
    fft64_inplace(x);
    if constexpr (EQ) {
      const uint32_t* cp = chan + (int64_t)p * 64;
      equalize_data_bins(x, [cp](int b) { return as_s2(cp[b]); }, 0, T);
    }
    demap_deinterleave<0>(x, lut, w);
  } else {
#pragma unroll
    for (int d = 0; d < 12; d++) w[d] = 0;
  }
  uint4* dst = sig_soft + (int64_t)p * 3;
  dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
  dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
  dst[2] = make_uint4(w[8], w[9], w[10], w[11]);
}

// ------------------------------------------------------------------ SIGNAL Viterbi (rows)
// Viterbi_sig11 (viterbicore.hpp:272-315) on the data Viterbi's row layout (zrx_viterbi3.hpp:
// a packet = one kLanes-lane row, v3::kRows packets a block): 24 rate-1/2 columns on the
// 48 soft values, normalize after columns 8, 16 and 24 (the reference's extra normalize after
// the loop is then a no-op: the metric minimum is 0 or 1), traceback of 24 bits with lookahead
// 0 from the key argmin.  parsePLCPHeader keeps bits 6..23 of the traceback word (the >> 6
// at sora_ext_viterbi.cpp:191), i.e. the decisions of columns 7..24: columns 23, 24 are the
// winner's newest pad bits, 15..22 and 7..14 the pad bytes stored at columns 22 and 14 (the
// column with cycle phase 7) along its path.  So a packet costs 24 packed columns of one row,
// two snapshots and two dependent LDS reads (tests/vit8_model.py signal_header_bits restates it).
// Rate-1/2 columns never wrap the u8 metric (zrx_viterbi3.hpp "Guard-free columns": the
// initial 0 / 48 metrics included), so they run without the guard.
__device__ __forceinline__ uint32_t sig_soft_byte(const uint32_t (&sw)[12], int i) {
  return sw[i >> 2] >> (8 * (i & 3));
}
template <int J>
__device__ __forceinline__ void sig_col(uint32_t (&M)[v3::kDw], const v3::Consts& K, const uint32_t (&sw)[12],
                                        uint8_t (*snap)[64], uint32_t l) {
  const uint32_t P = v3::p_word(v3::p_kind(0), sig_soft_byte(sw, 2 * J), sig_soft_byte(sw, 2 * J + 1));
  v3::column5<J % 6, 0, (J + 2) % 8, false>(M, P, K);
  constexpr int c = J + 1;                             // columns done
  if constexpr (c % 8 == 0) v3::normalize(M);
  if constexpr (c == 14 || c == 22) {                  // pad bytes by state (position p: rotl6(p, c))
#pragma unroll
    for (int q = 0; q < 2 * v3::kDw; q++)
      snap[c == 22][v3::rotl6(v3::pos_of(l, q >> 1, q & 1), c % 6)] = (uint8_t)(M[q >> 1] >> (16 * (q & 1)));
  }
}
template <int... J>
__device__ __forceinline__ void sig_cols(uint32_t (&M)[v3::kDw], const v3::Consts& K, const uint32_t (&sw)[12],
                                         uint8_t (*snap)[64], uint32_t l, std::integer_sequence<int, J...>) {
  (sig_col<J>(M, K, sw, snap, l), ...);
}
// The 18 header bits (bits 6..23 of the sig11 traceback word) of the row's packet.
__device__ __forceinline__ uint32_t sig_header_bits(const uint32_t (&sw)[12], uint32_t l, uint8_t (*snap)[64]) {
  v3::Consts K;
  v3::make_consts(K, l, 0);
  uint32_t M[v3::kDw];
#pragma unroll
  for (int d = 0; d < v3::kDw; d++)                    // H = 0 at state 0, 48 elsewhere (halved, bits 14..8)
    M[d] = (v3::pos_of(l, d, 0) ? 24u << 8 : 0u) | ((v3::pos_of(l, d, 1) ? 24u << 8 : 0u) << 16);
  sig_cols(M, K, sw, snap, l, std::make_integer_sequence<int, 24>{});
  // argmin of the signed int16 key (m << 8) | 4s at column 24 (24 mod 6 = 0: state = position),
  // m = the reference's metric: H | the marker of column 24 (pad bit 1)
  uint32_t best = 0xFFFFFFFFu;
#pragma unroll
  for (int q = 0; q < 2 * v3::kDw; q++) {
    const uint32_t half = (M[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
    const uint32_t m = ((half >> 7) & 0xFEu) | ((half >> 1) & 1u);
    const uint32_t ukey = (((m << 8) | (v3::pos_of(l, q >> 1, q & 1) << 2)) & 0xFFFFu) ^ 0x8000u;
    best = min(best, (ukey << 16) | (half & 3u));
  }
  best = min(best, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)best, 0xB1, 0xF, 0xF, false));
  best = min(best, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)best, 0x4E, 0xF, 0xF, false));
  if constexpr (v3::kLanes >= 8) best = min(best, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)best, 0x141, 0xF, 0xF, false));
  if constexpr (v3::kLanes == 16) best = min(best, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)best, 0x140, 0xF, 0xF, false));
  const uint32_t s0 = (best >> 18) & 63u, pad = best & 3u;   // pad bit 0: column 23, bit 1: column 24
  // state at column 22: its bits 0..3 = s0 bits 2..5, bit 4 = decision 24, bit 5 = decision 23
  const uint32_t s22 = (s0 >> 2) | ((pad >> 1) << 4) | ((pad & 1u) << 5);
  const uint32_t b22 = snap[1][s22];                   // decisions of columns 15..22 (bit j: 15 + j)
  const uint32_t b14 = snap[0][v3::rev6(b22 & 63u)];   // columns 7..14; state at 14 = rev6(decisions 15..20)
  return b14 | (b22 << 8) | (pad << 16);
}

__device__ __forceinline__ int ncbps_of(int mod) { return mod == 0 ? 48 : mod == 1 ? 96 : mod == 2 ? 192 : 288; }
// N_DBPS (transmitter.blk:39-46)
__device__ __forceinline__ int ndbps_of(int mod, int coding) {
  const int nc = ncbps_of(mod);
  return coding == 0 ? nc / 2 : coding == 1 ? nc * 2 / 3 : nc * 3 / 4;
}

// SIGNAL Viterbi + parsePLCPHeader -> Viterbi/FFT parameters and packet info.
// vparams[4p..] = {frame_len, code_rate, soft_len, modulation}
// info[8p..]    = {modulation, coding, len, header_err, crc_ok, status, symbols_used, viterbi_bits}
// cap_nsym: symbols per packet the soft workspace holds (zrx_reserve); a packet whose header
// asks for more gets ZRX_PKT_OVERSIZE and no soft values, so nothing writes past its slot.
// plan (the rx chain's plan header, or null): a packet that asks for something else than the
// uniform batch of npkts packets the last plan described raises kPlanMismatch (k_pkt_plan).
__global__ __launch_bounds__(256) void k_signal_vit(const uint32_t* __restrict__ sig_soft, const int32_t* __restrict__ nsym,
                                                    int npkts, int cap_nsym, int32_t* __restrict__ vparams,
                                                    int32_t* __restrict__ info, int32_t* plan) {
  __shared__ uint8_t snap[v3::kRows][2][64];           // [row][column 14, 22][state]
  const uint32_t l = threadIdx.x & (v3::kLanes - 1u), r = threadIdx.x >> v3::kLaneBits;
  const int wave0 = blockIdx.x * v3::kRows + (int)((threadIdx.x >> 6) * v3::kRowsWave);
  if (wave0 >= npkts) return;                          // (wave-uniform)
  const int p = blockIdx.x * v3::kRows + (int)r;
  const uint4* src = (const uint4*)(sig_soft + (int64_t)min(p, npkts - 1) * 12);
  const uint4 q0 = src[0], q1 = src[1], q2 = src[2];
  const uint32_t sw[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
  const uint32_t hb = sig_header_bits(sw, l, snap[r]);
  if (p >= npkts) return;
  // parsePLCPHeader.blk:124-158 RATE nibble (bit k of the nibble = hdata[k])
  int mod = 0, cod = 0;
  switch (hb & 0xF) {
    case 0xB: mod = 0; cod = 0; break;
    case 0xF: mod = 0; cod = 2; break;
    case 0xA: mod = 1; cod = 0; break;
    case 0xE: mod = 1; cod = 2; break;
    case 0x9: mod = 2; cod = 0; break;
    case 0xD: mod = 2; cod = 2; break;
    case 0x8: mod = 3; cod = 1; break;
    case 0xC: mod = 3; cod = 2; break;
    default: mod = 0; cod = 0;
  }
  int len = (int)((hb >> 5) & 0xFFF);
  int err = 0;
  if (len > 2048) { err = 1; len = 2048; }            // :171-174
  if (__builtin_popcount(hb) & 1) err = 1;            // parity over 24 bits (:177-188)
  const int nd = ndbps_of(mod, cod);
  const int need = (16 + 8 * len + 6 + nd - 1) / nd;  // symbols holding SERVICE .. tail
  int status = 0;
  if (err) status = 1;
  else if (need > nsym[p] - 1) status = 2;
  else if (need > cap_nsym - 1) status = 3;
  if (l == 0) {
    int32_t* vp = vparams + 4 * (int64_t)p;
    vp[0] = len + 2;                                  // Decode.blk:59 Viterbi(h.coding, h.len+2)
    vp[1] = cod;
    vp[2] = status == 0 ? need * ncbps_of(mod) : 0;
    vp[3] = mod;
    int32_t* in = info + 8 * (int64_t)p;
    in[0] = mod; in[1] = cod; in[2] = len; in[3] = err; in[4] = 0; in[5] = status;
    in[6] = 1 + (status == 0 ? need : 0); in[7] = 0;
    if (plan && plan[v3::kPlanExpN] == npkts &&
        (plan[v3::kPlanExpLen] != vp[0] || plan[v3::kPlanExpCr] != vp[1] || plan[v3::kPlanExpSoft] != vp[2] ||
         plan[v3::kPlanExpMod] != vp[3]) &&
        *(volatile int32_t*)(plan + v3::kPlanMismatch) == 0)   // (once raised, no more atomics)
      atomicOr(plan + v3::kPlanMismatch, 1);
  }
}

// The per-batch plan, from what each packet's header asks for (vparams, k_signal_vit), in
// one kernel right after it:
//   off[p]       = sum over q < p of soft_len(q) rounded up to 256 B (packed soft slots: a
//                  batch's soft values stay within the Viterbi's 4 GiB read window, which a
//                  mixed batch sized for its longest packet at 64-QAM would not);
//   dsym[p]      = sum over q < p of the data symbols of q; dsym[npkts] = all of them;
//   wave_p0[w]   = the packet holding batch data symbol 64w (k_data_fft's waves);
//   rows, nrows  = k_viterbi3's row table when rows is not null: every packet cut into
//                  segs[p] trellis segments (zrx_viterbi3.hpp) of about L columns, L = the
//                  batch's columns / (64 rows per CU x ncu), so a batch of few or unequal
//                  frames still gives every SIMD four waves (a batch of equal frames that
//                  already does, e.g. BASELINE config 3, is not cut); the rows ordered by
//                  (rate, segment length) — the segments of a packet on consecutive rows —
//                  and placed snake over the CUs; a packet with no trellis columns (header
//                  error, truncated) gets no row and out_bits[p] = 0.  order[]: scratch.
// off null: rows only (the Viterbi device API, whose soft offsets are the caller's).
// One 1024-thread block, rounds of 16 x 1024 packets: every thread loads its 16 packets'
// parameters (p = round base + 1024 i + thread: coalesced, all loads in flight together),
// 16 independent DPP wave scans of the two 32-bit sums (256-B units, symbols), one table of
// 256 (chunk, wave) offsets scanned by wave 0, every thread's 16 offsets from it; then the
// segment length from the batch's column total, the packet keys counted in one pass and
// scattered in another, and the rows expanded from the sorted packets by a block scan.
constexpr int kScanPer = 16;
#ifndef ZRX_RANK_BLOCKS
#define ZRX_RANK_BLOCKS 1   // (0: A/B builds without the ranked block placement)
#endif
#ifndef ZRX_PLAN_CUT
#define ZRX_PLAN_CUT 99   // (scripts/ubench/plan_ubench.hip: time k_pkt_plan up to one of its phases)
#endif
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);   // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);   // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);   // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);   // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}
// Packets in row order: every packet with trellis columns is cut into nseg segments
// (v3::seg_count) and keyed by (rate, segment length); the counting pass writes segs[p] (and
// out_bits[p] = 0 for a packet with no columns, which gets no row) and counts keys and rows,
// the scatter pass writes order[] (packets sorted by key).
template <bool SCATTER>
__device__ __forceinline__ void plan_pkts(const int32_t* __restrict__ vparams, int npkts, uint32_t L, uint32_t* hist,
                                          int32_t* __restrict__ order, uint8_t* __restrict__ segs,
                                          int32_t* __restrict__ out_bits, uint32_t* nrows_total) {
  const int t = threadIdx.x;
  uint32_t my_rows = 0;
  for (int base = 0; base < npkts; base += 1024 * kScanPer) {
    int4 q[kScanPer];
#pragma unroll
    for (int i = 0; i < kScanPer; i++) {
      const int p = base + 1024 * i + t;
      q[i] = p < npkts ? *reinterpret_cast<const int4*>(vparams + 4 * (int64_t)p) : make_int4(0, -1, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < kScanPer; i++) {
      const int p = base + 1024 * i + t;
      const bool valid = p < npkts;
      const uint32_t cols = cols_of(q[i].y, q[i].z);
      const uint32_t E = q[i].x < 0 || q[i].x > (1 << 21) ? 0xFFFFFFFFu : (uint32_t)q[i].x * 8u + 6u;
      const uint32_t nseg = SCATTER ? (valid ? (uint32_t)segs[p] : 0u) : cols ? v3::seg_count(E, cols, L) : 0u;
      if (!SCATTER && valid) {
        segs[p] = (uint8_t)nseg;
        if (nseg == 0) out_bits[p] = 0;
        my_rows += nseg;
      }
      // segment length: about cols / nseg, plus the seam overlap
      const uint32_t len = nseg <= 1u ? cols : v3::udiv_small(min(cols, (1u << 20) - 1u) + nseg - 1u, nseg) + 286u;
      const uint32_t slot = order_claim(hist, valid && nseg > 0u, order_key_len(q[i].y, len));
      if (SCATTER && valid && nseg > 0u) order[slot] = p;
    }
  }
  if (!SCATTER) {
    for (int o = 32; o > 0; o >>= 1) my_rows += (uint32_t)__shfl_xor((int)my_rows, o);
    if ((t & 63) == 0) atomicAdd(nrows_total, my_rows);
  }
}
// The mixed batch's rows (k_pkt_plan's comment): packets keyed by (rate, segment length)
// with segment length Lm, counted and scattered in LDS (hist: kOrderPerThread x 1024 words,
// zeroed; *rtotal zeroed), then expanded onto rows by a block scan.  1024 threads.
// (Ranked placement, interleaved A/B on config 5: Viterbi 0.637-0.648 -> 0.597-0.629 ms; an
// earlier version that re-ranked waves and blocks inside the snake measured 0.672 -> 0.75.)
__device__ __forceinline__ void plan_rows_mixed(const int32_t* __restrict__ vparams, int npkts, uint32_t Lm,
                                                int2* __restrict__ rows, int32_t* __restrict__ nrows,
                                                uint8_t* __restrict__ segs, int32_t* __restrict__ order,
                                                int32_t* __restrict__ out_bits, int ncu, int rows_cap, uint32_t* hist,
                                                uint32_t* rtotal) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  plan_pkts<false>(vparams, npkts, Lm, hist, order, segs, out_bits, rtotal);
  __syncthreads();
  if (ZRX_PLAN_CUT <= 3) return;
  const uint32_t npk = order_hist_scan(hist);          // packets with rows
  __syncthreads();
  plan_pkts<true>(vparams, npkts, Lm, hist, order, segs, out_bits, nullptr);
  __syncthreads();                                     // order[] and segs[] written by the block
  if (ZRX_PLAN_CUT <= 5) return;
  // Expand: the segments of the packet at sorted position i are rows prefix(i) .. +nseg - 1
  // (consecutive, so a wave holds segments of one or two packets of similar length).  Thread
  // t takes positions 16t .. 16t + 15 of each round.  Two sweeps: the first finds each whole
  // block's longest row (blk[]), the blocks are ranked by it and placed (v3::rank_place), and
  // the second writes the rows there.  (Sorted by rate first, the blocks' lengths rise and
  // fall three times, and the snake over that order paired long blocks with long ones: config
  // 5's per-SIMD columns spread 768..11 614 around a mean of 9026.)
  // (ranked units: kPlanUnit rows, a block's 32, placed over the CUs)
  const uint32_t total = *rtotal, nfull = total / (uint32_t)v3::kPlanUnit;
  const uint32_t ncu2 = (uint32_t)max(ncu, 2), ncu_rcp = 0xFFFFFFFFu / ncu2 + 1u;
  const bool ranked = ZRX_RANK_BLOCKS && nfull <= (uint32_t)v3::kRankBlocks;
  __shared__ uint32_t esum[16];
  __shared__ uint32_t blk[v3::kRankBlocks];           // longest row, then the placed slot
  if (ranked)
    for (uint32_t b = t; b < nfull; b += 1024u) blk[b] = 0u;
  __syncthreads();
  for (int sweep = ranked ? 0 : 1; sweep < 2; sweep++) {
    uint32_t carry = 0;
    for (uint32_t base = 0; base < npk; base += 1024u * kScanPer) {
      int32_t pk[kScanPer];
      uint32_t ns[kScanPer], sum = 0;
#pragma unroll
      for (int i = 0; i < kScanPer; i++) {
        const uint32_t pos = base + kScanPer * (uint32_t)t + i;
        pk[i] = pos < npk ? order[pos] : -1;
      }
#pragma unroll
      for (int i = 0; i < kScanPer; i++) { ns[i] = pk[i] >= 0 ? segs[pk[i]] : 0u; sum += ns[i]; }
      const uint32_t inc = wave_incl_scan(sum);
      if (lane == 63) esum[wv] = inc;
      __syncthreads();
      uint32_t ex = carry + inc - sum, rnd = 0;
      for (int w = 0; w < 16; w++) { ex += w < wv ? esum[w] : 0u; rnd += esum[w]; }
#pragma unroll
      for (int i = 0; i < kScanPer; i++) {
        if (sweep == 0) {
          if (ns[i] != 0u) {                           // the row length the sort keyed on
            const int4 q = *reinterpret_cast<const int4*>(vparams + 4 * (int64_t)pk[i]);
            const uint32_t cols = cols_of(q.y, q.z);
            const uint32_t len = ns[i] <= 1u ? cols : v3::udiv_small(min(cols, (1u << 20) - 1u) + ns[i] - 1u, ns[i]) + 286u;
            for (uint32_t b = ex / (uint32_t)v3::kPlanUnit; b * (uint32_t)v3::kPlanUnit < ex + ns[i] && b < nfull; b++)
              atomicMax(&blk[b], len);
          }
        } else {
          for (uint32_t k = 0; k < ns[i]; k++) {
            const uint32_t pos = ex + k, b = pos / (uint32_t)v3::kPlanUnit;
            const uint32_t at = !ranked ? v3::order_place(pos, nfull, ncu2, ncu_rcp)
                                : b < nfull ? blk[b] * (uint32_t)v3::kPlanUnit + pos % (uint32_t)v3::kPlanUnit : pos;
            if (at < (uint32_t)rows_cap) rows[at] = make_int2(pk[i], (int)(k | (ns[i] << 8)));   // (always: the plan's row bound)
          }
        }
        ex += ns[i];
      }
      carry += rnd;
      __syncthreads();                                 // esum is rewritten by the next round
    }
    if (sweep == 0) {
      // rank the whole blocks by their longest row, longest first (a counting sort over
      // 24-column bodies in hist[0 .. 1023]; ties in any order), then place them
      for (int i = t; i < kOrderPerThread * 1024; i += 1024) hist[i] = 0;
      __syncthreads();
      for (uint32_t b0 = 0; b0 < nfull; b0 += 1024u) {
        const uint32_t b = b0 + (uint32_t)t;
        const uint32_t key = b < nfull ? (uint32_t)kOrderLen - 1u - min((blk[b] + 23u) / 24u, (uint32_t)kOrderLen - 1u) : 0u;
        if (b < nfull) atomicAdd(&hist[key], 1u);
      }
      __syncthreads();
      order_hist_scan(hist);
      __syncthreads();
      for (uint32_t b0 = 0; b0 < nfull; b0 += 1024u) {
        const uint32_t b = b0 + (uint32_t)t;
        const uint32_t key = b < nfull ? (uint32_t)kOrderLen - 1u - min((blk[b] + 23u) / 24u, (uint32_t)kOrderLen - 1u) : 0u;
        const uint32_t r = order_claim(hist, b < nfull, key);
        __syncthreads();                               // every lane read blk[] before it is rewritten
        if (b < nfull) blk[b] = v3::rank_place(r, nfull, ncu2, ncu_rcp);
      }
      __syncthreads();
    }
  }
  if (t == 0) {
    nrows[v3::kPlanRows] = (int32_t)min(total, (uint32_t)rows_cap);
    nrows[v3::kPlanFixes] = 0;                         // counted by the seam pass
    nrows[v3::kPlanUniform] = 0;
    // rows past the bound (plan_rows_max) are dropped: never by construction, but a wrong
    // bound must show (zrx_plan_check) instead of leaving packets silently undecoded
    nrows[v3::kPlanDropped] = total > (uint32_t)rows_cap ? (int32_t)(total - (uint32_t)rows_cap) : 0;
    nrows[v3::kPlanNcu] = (int32_t)ncu2;
  }
}

__global__ __launch_bounds__(1024) void k_pkt_plan(const int32_t* __restrict__ vparams, int npkts,
                                                   int64_t* __restrict__ off, int32_t* __restrict__ dsym,
                                                   int32_t* __restrict__ wave_p0, int2* __restrict__ rows,
                                                   int32_t* __restrict__ nrows, uint8_t* __restrict__ segs,
                                                   int32_t* __restrict__ order, int32_t* __restrict__ out_bits, int ncu,
                                                   int rows_cap, int split, int32_t* __restrict__ mixed_hint) {
  __shared__ uint2 wtab[kScanPer * 16];                // (chunk i, wave w) totals, then offsets
  __shared__ uint2 round_total;
  __shared__ uint32_t hist[kOrderPerThread * 1024];
  __shared__ unsigned long long tcols;
  __shared__ uint32_t rtotal, uniform, reuse;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // The rx chain's batch equals the uniform batch the last plan described (k_signal_vit raised
  // no mismatch): offsets, wave starts and the row header are all still right.  Otherwise the
  // plan is rebuilt and forgets the old batch first.
  if (t == 0) {
    reuse = off && rows && nrows[v3::kPlanExpN] == npkts && nrows[v3::kPlanMismatch] == 0;
    if (reuse) {
      nrows[v3::kPlanFixes] = 0;                       // (counted afresh by this launch's seam pass)
    } else {
      nrows[v3::kPlanExpN] = 0;
      nrows[v3::kPlanMismatch] = 0;
    }
  }
  __syncthreads();
  if (reuse) return;
  if (rows) {
    for (int i = t; i < kOrderPerThread * 1024; i += 1024) hist[i] = 0;
    if (t == 0) { tcols = 0; rtotal = 0; uniform = 1; }
    __syncthreads();
  }
  uint64_t carry_u = 0;                                // 256-B units before this round
  uint32_t carry_s = 0;                                // symbols before this round
  uint64_t my_cols = 0;                                // trellis columns of this thread's packets
  // a uniform batch: every packet asks for the same frame length, rate and soft count
  const int4 q0 = npkts > 0 ? *reinterpret_cast<const int4*>(vparams) : make_int4(0, 0, 0, 0);
  bool same = cols_of(q0.y, q0.z) > 0;
  for (int base = 0; base < npkts; base += 1024 * kScanPer) {
    uint32_t vu[kScanPer], vs[kScanPer], iu[kScanPer], is[kScanPer];
#pragma unroll
    for (int i = 0; i < kScanPer; i++) {
      const int p = base + 1024 * i + t;
      vu[i] = vs[i] = 0;
      if (p < npkts) {
        const int4 q = *reinterpret_cast<const int4*>(vparams + 4 * (int64_t)p);   // {frame_len, cr, soft_len, mod}
        const uint32_t n = (uint32_t)max(q.z, 0);
        vu[i] = (n + 255u) >> 8;
        vs[i] = q.w == 3 ? n / 288u : (n >> (q.w & 3)) / 48u;   // soft_len / N_CBPS, constant divisors
        my_cols += cols_of(q.y, q.z);
        same = same && q.x == q0.x && q.y == q0.y && q.z == q0.z && q.w == q0.w;
      }
    }
    if (!off) continue;
#pragma unroll
    for (int i = 0; i < kScanPer; i++) { iu[i] = wave_incl_scan(vu[i]); is[i] = wave_incl_scan(vs[i]); }
    if (lane == 63) {
#pragma unroll
      for (int i = 0; i < kScanPer; i++) wtab[16 * i + wv] = make_uint2(iu[i], is[i]);
    }
    __syncthreads();
    if (wv == 0) {                                     // exclusive scan of the 256 totals, 4 per lane
      uint2 x[4];
      uint32_t su = 0, ss = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) { x[j] = wtab[4 * lane + j]; su += x[j].x; ss += x[j].y; }
      uint32_t eu = wave_incl_scan(su) - su, es = wave_incl_scan(ss) - ss;
#pragma unroll
      for (int j = 0; j < 4; j++) { wtab[4 * lane + j] = make_uint2(eu, es); eu += x[j].x; es += x[j].y; }
      if (lane == 63) round_total = make_uint2(eu, es);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kScanPer; i++) {
      const int p = base + 1024 * i + t;
      if (p < npkts) {
        const uint2 e = wtab[16 * i + wv];
        const uint64_t u0 = carry_u + e.x + iu[i] - vu[i];
        const uint32_t s0 = carry_s + e.y + is[i] - vs[i], s1 = s0 + vs[i];
        off[p] = (int64_t)(u0 << 8);
        dsym[p] = (int32_t)s0;
        for (uint32_t w = (s0 + 63u) >> 6; 64u * w < s1; w++) wave_p0[w] = p;
      }
    }
    const uint2 rt = round_total;
    carry_u += rt.x;
    carry_s += rt.y;
    __syncthreads();                                   // wtab is rewritten by the next round
  }
  if (off && t == 0) dsym[npkts] = (int32_t)carry_s;   // the whole batch's data symbols
  if (!rows || ZRX_PLAN_CUT <= 1) return;
  for (int o = 32; o > 0; o >>= 1) my_cols += (uint64_t)__shfl_xor((long long)my_cols, o);
  if (lane == 0) atomicAdd(&tcols, (unsigned long long)my_cols);
  if (!same) uniform = 0;
  __syncthreads();
  const uint64_t rt = 64ull * (uint64_t)max(ncu, 1);   // rows that give every SIMD four waves
  const uint32_t L0 = (uint32_t)min<uint64_t>((tcols + rt - 1) / rt, 0xFFFFFFFFull);
  const uint32_t L = max(L0, v3::kMinSeg);
  // (a frame is cut only when it is more than L + L / 8 long: a batch of equal frames just
  // short of four waves per SIMD stays whole; a small uniform batch down to kMinCut)
  const uint32_t Lu = max(L0, v3::kMinCut);
  const uint32_t Lb = Lu + Lu / 8u;                     // (uniform batch)
  const uint32_t Lm = max(L * v3::kSegMixNum / 8u, v3::kMinSeg);   // (mixed batch)
  if (t == 0 && mixed_hint) *mixed_hint = uniform ? 0 : 1;   // (host-mapped: the next call's split choice)
  if (uniform) {                                       // no sort: k_viterbi3 derives each row's segment
    if (t == 0) {
      const uint32_t E0 = q0.x > (1 << 21) ? 0xFFFFFFFFu : (uint32_t)q0.x * 8u + 6u;
      const uint32_t n0 = v3::seg_count(E0, cols_of(q0.y, q0.z), Lb, v3::kMinCut);
      nrows[v3::kPlanRows] = (int32_t)min((uint32_t)npkts * n0, (uint32_t)rows_cap);
      nrows[v3::kPlanFixes] = 0;
      nrows[v3::kPlanUniform] = (int32_t)n0;
      nrows[v3::kPlanDropped] = (uint32_t)npkts * n0 > (uint32_t)rows_cap ? (int32_t)((uint32_t)npkts * n0 - rows_cap) : 0;
      nrows[v3::kPlanNcu] = ncu;
      if (off) {                                       // the batch a next launch may reuse this plan for
        nrows[v3::kPlanExpLen] = q0.x; nrows[v3::kPlanExpCr] = q0.y;
        nrows[v3::kPlanExpSoft] = q0.z; nrows[v3::kPlanExpMod] = q0.w;
        nrows[v3::kPlanExpN] = npkts;
      }
    }
    return;
  }
  if (split) {                                         // k_pkt_rows sorts and expands, on a side stream
    if (t == 0) nrows[v3::kPlanUniform] = 0;            // (k_pkt_rows writes the same)
    return;
  }
  plan_rows_mixed(vparams, npkts, Lm, rows, nrows, segs, order, out_bits, ncu, rows_cap, hist, &rtotal);
}

// ---- k_pkt_scan: the rx chain's plan over many blocks ------------------------------------
// k_pkt_plan's offsets scan (off, dsym, wave_p0) and its batch verdict (uniform or mixed:
// the mixed-batch hint, the uniform plan header, a mixed batch's rows) in one launch of
// ceil(npkts / 4096) blocks instead of one block's chain of dependent rounds (config 5: 28 us
// on the head's critical path).  Each block takes 4096 consecutive packets (4 a thread),
// publishes its sums (256-B soft units, data symbols, trellis columns, all-equal flag) in
// rec[block] with the launch's epoch as the ready mark, adds the published sums of every block
// before it (those were dispatched earlier and publish without waiting on anything, so the
// spin always ends) and writes its packets' offsets.  The last block to finish (a counter it
// resets) reduces the records and plans as k_pkt_plan did: the uniform header, or a mixed
// batch's rows (plan_rows_mixed) unless k_pkt_rows does them beside k_data_fft (split).
// nrows null: offsets only.
constexpr int kPsThreads = 1024, kPsPer = 4, kPsBlock = kPsThreads * kPsPer;
// A block's record: three self-validating words, each {epoch, value} written by one 64-bit
// relaxed atomic store and read by relaxed atomic loads (which the memory model keeps coherent
// across the XCDs' L2s) until the epoch matches, so no release / acquire fence is needed (an
// agent-scope fence writes back or invalidates the XCD's whole L2).
struct PlanScanRec {
  unsigned long long wu, ws, wc;   // epoch << 32 | 256-B soft units; | data symbols; | same << 31 | columns
};
__device__ __forceinline__ unsigned long long ps_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ps_store(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// spin until a record word carries this launch's epoch; its value
__device__ __forceinline__ uint32_t ps_wait(const unsigned long long* p, uint32_t epoch) {
  unsigned long long v;
  while ((uint32_t)((v = ps_load(p)) >> 32) != epoch) __builtin_amdgcn_s_sleep(1);
  return (uint32_t)v;
}
__global__ __launch_bounds__(kPsThreads) void k_pkt_scan(const int32_t* __restrict__ vparams, int npkts,
                                                         int64_t* __restrict__ off, int32_t* __restrict__ dsym,
                                                         int32_t* __restrict__ wave_p0, int2* __restrict__ rows,
                                                         int32_t* __restrict__ nrows, uint8_t* __restrict__ segs,
                                                         int32_t* __restrict__ order, int32_t* __restrict__ out_bits,
                                                         int ncu, int rows_cap, int split,
                                                         int32_t* __restrict__ mixed_hint,
                                                         PlanScanRec* __restrict__ rec, uint32_t* __restrict__ ctr,
                                                         uint32_t epoch) {
  constexpr int kW = kPsThreads / 64;
  __shared__ uint32_t wsum_u[kW], wsum_s[kW], wflag[kW];
  __shared__ unsigned long long wcols[kW];
  __shared__ uint32_t pre_u, pre_s, last, rtotal;
  __shared__ uint32_t hist[kOrderPerThread * 1024];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, b = blockIdx.x, nb = gridDim.x;
  if (nrows) {
    // (the reuse test of k_pkt_plan: every block reads the same words, and block 0 changes them
    // only to values that make every later reader decide the same way)
    const bool reuse = nrows[v3::kPlanExpN] == npkts && nrows[v3::kPlanMismatch] == 0;
    if (reuse) {
      if (b == 0 && t == 0) nrows[v3::kPlanFixes] = 0;
      return;
    }
    if (b == 0 && t == 0) { nrows[v3::kPlanExpN] = 0; nrows[v3::kPlanMismatch] = 0; }
  }
  const int4 q0 = *reinterpret_cast<const int4*>(vparams);
  const int p0 = b * kPsBlock + kPsPer * t;
  uint32_t vu[kPsPer], vs[kPsPer], su = 0, ss = 0;
  uint64_t my_cols = 0;
  bool same = cols_of(q0.y, q0.z) > 0;
#pragma unroll
  for (int i = 0; i < kPsPer; i++) {
    vu[i] = vs[i] = 0;
    const int p = p0 + i;
    if (p < npkts) {
      const int4 q = *reinterpret_cast<const int4*>(vparams + 4 * (int64_t)p);   // {frame_len, cr, soft_len, mod}
      const uint32_t n = (uint32_t)max(q.z, 0);
      vu[i] = (n + 255u) >> 8;
      vs[i] = q.w == 3 ? n / 288u : (n >> (q.w & 3)) / 48u;   // soft_len / N_CBPS
      my_cols += cols_of(q.y, q.z);
      same = same && q.x == q0.x && q.y == q0.y && q.z == q0.z && q.w == q0.w;
    }
    su += vu[i];
    ss += vs[i];
  }
  // block scan of the threads' sums; the block's totals
  const uint32_t iu = wave_incl_scan(su), is = wave_incl_scan(ss);
  for (int o = 32; o > 0; o >>= 1) my_cols += (uint64_t)__shfl_xor((long long)my_cols, o);
  const bool wsame = __builtin_amdgcn_ballot_w64(!same) == 0ull;
  if (lane == 63) { wsum_u[wv] = iu; wsum_s[wv] = is; }
  if (lane == 0) { wcols[wv] = my_cols; wflag[wv] = wsame ? 1u : 0u; }
  __syncthreads();
  uint32_t eu = iu - su, es = is - ss;
  for (int w = 0; w < wv; w++) { eu += wsum_u[w]; es += wsum_s[w]; }
  if (t == 0) {                                        // publish
    uint32_t bu = 0, bs = 0, bf = 1;
    unsigned long long bc = 0;
    for (int w = 0; w < kW; w++) { bu += wsum_u[w]; bs += wsum_s[w]; bc += wcols[w]; bf &= wflag[w]; }
    const unsigned long long e = (unsigned long long)epoch << 32;
    ps_store(&rec[b].wu, e | bu);
    ps_store(&rec[b].ws, e | bs);
    // (a block's columns: at most 4096 x 16406 < 2^31)
    ps_store(&rec[b].wc, e | ((unsigned long long)bf << 31) | (bc & 0x7FFFFFFFull));
  }
  if (wv == 0) {                                       // every earlier block's sums
    uint32_t au = 0, as = 0;
    for (int j0 = 0; j0 < b; j0 += 64) {
      const int j = j0 + lane;
      if (j < b) {
        au += ps_wait(&rec[j].wu, epoch);
        as += ps_wait(&rec[j].ws, epoch);
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      au += (uint32_t)__shfl_xor((int)au, o);
      as += (uint32_t)__shfl_xor((int)as, o);
    }
    if (lane == 0) { pre_u = au; pre_s = as; }
  }
  __syncthreads();
  uint64_t u0 = (uint64_t)pre_u + eu;
  uint32_t s0 = pre_s + es;
#pragma unroll
  for (int i = 0; i < kPsPer; i++) {
    const int p = p0 + i;
    if (p < npkts) {
      off[p] = (int64_t)(u0 << 8);
      dsym[p] = (int32_t)s0;
      for (uint32_t w = (s0 + 63u) >> 6; 64u * w < s0 + vs[i]; w++) wave_p0[w] = p;
    }
    u0 += vu[i];
    s0 += vs[i];
  }
  // the last block to get here reduces the records (each read as its epoch shows it): the
  // batch's totals and its verdict
  if (t == 0) {
    last = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)nb - 1u;
    if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // (for the next launch)
  }
  __syncthreads();
  if (!last) return;
  uint64_t tc = 0;
  uint32_t ts = 0, all_same = 1;
  for (int j = t; j < nb; j += kPsThreads) {
    const uint32_t c = ps_wait(&rec[j].wc, epoch);
    tc += c & 0x7FFFFFFFu;
    all_same &= c >> 31;
    ts += ps_wait(&rec[j].ws, epoch);
  }
  for (int o = 32; o > 0; o >>= 1) {
    tc += (uint64_t)__shfl_xor((long long)tc, o);
    ts += (uint32_t)__shfl_xor((int)ts, o);
  }
  const bool ws = __builtin_amdgcn_ballot_w64(all_same == 0u) == 0ull;
  __syncthreads();                                     // (the block's sums above were read)
  if (lane == 0) { wcols[wv] = tc; wsum_s[wv] = ts; wflag[wv] = ws ? 1u : 0u; }
  __syncthreads();
  uint64_t tcols = 0;
  uint32_t tsym = 0;
  bool uniform = true;
  for (int w = 0; w < kW; w++) { tcols += wcols[w]; tsym += wsum_s[w]; uniform = uniform && wflag[w]; }
  if (t == 0) dsym[npkts] = (int32_t)tsym;             // the whole batch's data symbols
  if (!nrows) return;
  if (t == 0 && mixed_hint) *mixed_hint = uniform ? 0 : 1;   // (host-mapped: the next call's split choice)
  const uint64_t rt = 64ull * (uint64_t)max(ncu, 1);   // rows that give every SIMD four waves
  const uint32_t L0 = (uint32_t)min<uint64_t>((tcols + rt - 1) / rt, 0xFFFFFFFFull);
  if (!uniform) {
    if (split) {
      if (t == 0) nrows[v3::kPlanUniform] = 0;         // (k_pkt_rows writes the same, beside k_data_fft)
      return;
    }
    for (int i = t; i < kOrderPerThread * 1024; i += kPsThreads) hist[i] = 0;
    if (t == 0) rtotal = 0;
    __syncthreads();
    const uint32_t L = max(L0, v3::kMinSeg);
    const uint32_t Lm = max(L * v3::kSegMixNum / 8u, v3::kMinSeg);
    plan_rows_mixed(vparams, npkts, Lm, rows, nrows, segs, order, out_bits, ncu, rows_cap, hist, &rtotal);
    return;
  }
  if (t != 0) return;
  const uint32_t Lu = max(L0, v3::kMinCut);            // k_pkt_plan's uniform header
  const uint32_t Lb = Lu + Lu / 8u;
  const uint32_t E0 = q0.x > (1 << 21) ? 0xFFFFFFFFu : (uint32_t)q0.x * 8u + 6u;
  const uint32_t n0 = v3::seg_count(E0, cols_of(q0.y, q0.z), Lb, v3::kMinCut);
  nrows[v3::kPlanRows] = (int32_t)min((uint32_t)npkts * n0, (uint32_t)rows_cap);
  nrows[v3::kPlanFixes] = 0;
  nrows[v3::kPlanUniform] = (int32_t)n0;
  nrows[v3::kPlanDropped] = (uint32_t)npkts * n0 > (uint32_t)rows_cap ? (int32_t)((uint32_t)npkts * n0 - rows_cap) : 0;
  nrows[v3::kPlanNcu] = ncu;
  nrows[v3::kPlanExpLen] = q0.x; nrows[v3::kPlanExpCr] = q0.y;
  nrows[v3::kPlanExpSoft] = q0.z; nrows[v3::kPlanExpMod] = q0.w;
  nrows[v3::kPlanExpN] = npkts;
}

// The second half of a split plan (rx chain): the mixed batch's sort and row expansion, on a
// side stream forked right after k_signal_vit, so it runs beside k_pkt_plan and k_data_fft
// (one block of 1024 threads: config 5's takes ~140 us, longer than k_data_fft alone).  It
// needs only the packets' parameters: the batch's column total (for the segment length) and
// whether it is uniform are recounted here exactly as k_pkt_plan counts them (one more read of
// 16 B per packet), so the two kernels share no state but the header words they both write
// with equal values.  Nothing to do for a uniform batch: k_pkt_plan writes its header.
__global__ __launch_bounds__(1024) void k_pkt_rows(const int32_t* __restrict__ vparams, int npkts,
                                                   int2* __restrict__ rows, int32_t* __restrict__ nrows,
                                                   uint8_t* __restrict__ segs, int32_t* __restrict__ order,
                                                   int32_t* __restrict__ out_bits, int ncu, int rows_cap) {
  __shared__ uint32_t hist[kOrderPerThread * 1024];
  __shared__ uint32_t rtotal, uniform;
  __shared__ unsigned long long tcols;
  const int t = threadIdx.x;
  if (t == 0) { rtotal = 0; uniform = 1; tcols = 0; }
  for (int i = t; i < kOrderPerThread * 1024; i += 1024) hist[i] = 0;
  __syncthreads();
  // (k_pkt_plan's rule: every packet asks for packet 0's {frame_len, rate, soft_len,
  // modulation} and it has trellis columns)
  const int4 q0 = npkts > 0 ? *reinterpret_cast<const int4*>(vparams) : make_int4(0, 0, 0, 0);
  bool same = cols_of(q0.y, q0.z) > 0;
  uint64_t my_cols = 0;
  for (int p = t; p < npkts; p += 1024) {
    const int4 q = *reinterpret_cast<const int4*>(vparams + 4 * (int64_t)p);
    my_cols += cols_of(q.y, q.z);
    same = same && q.x == q0.x && q.y == q0.y && q.z == q0.z && q.w == q0.w;
  }
  for (int o = 32; o > 0; o >>= 1) my_cols += (uint64_t)__shfl_xor((long long)my_cols, o);
  if ((t & 63) == 0) atomicAdd(&tcols, (unsigned long long)my_cols);
  if (!same) uniform = 0;
  __syncthreads();
  if (uniform) return;
  const uint64_t rt = 64ull * (uint64_t)max(ncu, 1);   // (k_pkt_plan's segment length Lm)
  const uint32_t L0 = (uint32_t)min<uint64_t>((tcols + rt - 1) / rt, 0xFFFFFFFFull);
  const uint32_t L = max(L0, v3::kMinSeg);
  const uint32_t Lm = max(L * v3::kSegMixNum / 8u, v3::kMinSeg);
  plan_rows_mixed(vparams, npkts, Lm, rows, nrows, segs, order, out_bits, ncu, rows_cap, hist, &rtotal);
}

// ---- k_data_fft: FFT64 + GetData + DemapLimit + Demap + Deinterleave, lane = data symbol ----
// The FFT runs one symbol per lane (no cross-lane traffic).  A lane's 288-B soft row is a poor
// store pattern (64 rows per store instruction), so each wave moves its rows through its own
// LDS region: the demapper writes unit q of the soft row to 19s + q (stride 19: the 8-lane
// groups of ds_write_b128 hit 8 slots), then 18 store instructions each take 64 consecutive
// units of the wave's rows, (s, q) = divmod(64j + lane, 18): 1 KiB runs.  A wave never waits
// on another: LDS is in order within a wave, so there are no barriers.  (Tried and dropped,
// PERFLOG.md: symbol loads by LDS-DMA, with and without a one-iteration prefetch; the next
// iteration's symbol prefetched into registers (233 VGPRs, 0.102 -> 0.110 ms); soft rows
// stored by each lane.)
#ifndef ZRX_DF_LUT_ONCE
#define ZRX_DF_LUT_ONCE 1
#endif
#ifndef ZRX_DF_WAVES
#define ZRX_DF_WAVES 4
#endif
#ifndef ZRX_DF_ROW
#define ZRX_DF_ROW 19
#endif
#ifndef ZRX_DF_LUTC
#define ZRX_DF_LUTC 4
#endif
constexpr int kDfWaves = ZRX_DF_WAVES;    // waves per block
constexpr int kDfThreads = 64 * kDfWaves;
constexpr int kDfRow = ZRX_DF_ROW;        // output staging row stride, 16-B units (a soft row is <= 18)
constexpr int kDfUnits = 64 * kDfRow;
constexpr int kDfLutCopies = ZRX_DF_LUTC; // demap LUT copies (lane & (copies - 1)): fewer LDS bank conflicts
static_assert(kDfRow >= 18 && (kDfLutCopies == 1 || kDfLutCopies == 2 || kDfLutCopies == 4) && 256 % kDfThreads == 0,
              "data FFT LDS layout");

__device__ __forceinline__ int soft_units_of(int mod) { return mod == 0 ? 3 : mod == 1 ? 6 : mod == 2 ? 12 : 18; }


// This lane's symbol of wave w: packet, index in the packet, modulation, symbol index, soft row.
struct DfSym {
  bool valid;
  int p, k, mod;
  uint32_t sidx, nu, obase;   // obase: soft row in 16-B units
};
// Where the lane's symbol g = 64w + lane sits (k_pkt_plan's numbering), from wave-uniform
// scalar loads: the wave's first packet wave_p0[w], then the packet boundaries dsym[q + 1 ..
// q + 8] eight at a time until a block passes the wave's last symbol (one block unless the
// wave spans more than 8 packets).  The per-lane loads of the packet's parameters are only
// issued here (df_finish waits for them), so the next wave's lookup runs under this one's FFT.
struct DfNext {
  bool valid;
  int p, k, mod;
  int64_t soff, ooff;
};
__device__ __forceinline__ void df_locate(int w, int lane, int total, int npkts, const int64_t* __restrict__ sym_off,
                                          const int32_t* __restrict__ vparams, const int64_t* __restrict__ soft_off,
                                          const int32_t* __restrict__ dsym, const int32_t* __restrict__ wave_p0,
                                          DfNext& n) {
  const int g = w * 64 + lane;
  n.valid = g < total;
  int q = __builtin_amdgcn_readfirstlane(wave_p0[w]);
  int p = q, base = dsym[q];
  const int glast = w * 64 + 63;
  for (;;) {
    int b[8];
#pragma unroll
    for (int j = 0; j < 8; j++) b[j] = dsym[min(q + 1 + j, npkts)];   // (dsym[npkts] = total)
#pragma unroll
    for (int j = 0; j < 8; j++)
      if (b[j] <= g) { p = q + 1 + j; base = b[j]; }
    if (b[7] > glast || q + 8 >= npkts) break;
    q += 8;
  }
  n.p = p;
  n.k = g - base;
  n.mod = n.valid ? vparams[4 * (int64_t)p + 3] : 0;
  n.soff = n.valid ? sym_off[p] : 0;
  n.ooff = n.valid ? soft_off[p] : 0;
}
__device__ __forceinline__ DfSym df_finish(const DfNext& n) {
  DfSym d;
  d.valid = n.valid;
  d.p = n.p;
  d.k = n.k;
  d.mod = n.mod;
  d.sidx = n.valid ? (uint32_t)(n.soff + 1 + n.k) : 0u;
  d.nu = n.valid ? (uint32_t)soft_units_of(n.mod) : 0u;
  d.obase = n.valid ? (uint32_t)(n.ooff / 16) + (uint32_t)n.k * d.nu : 0u;
  return d;
}

// Flat over the batch's data symbols (k_pkt_plan numbers them): wave w takes symbols
// 64w .. 64w+63, lane = symbol, whatever packets they belong to, so a long packet spreads
// over many waves and consecutive lanes write consecutive soft rows.  Waves loop over w with
// the grid's stride (the host sizes the grid from the call's max_nsym, an upper bound).
template <bool EQ>
__global__ __launch_bounds__(kDfThreads) void k_data_fft(const uint4* __restrict__ sym, const int64_t* __restrict__ sym_off,
                                                  const int32_t* __restrict__ vparams, int npkts,
                                                  uint4* __restrict__ soft, const int64_t* __restrict__ soft_off,
                                                  const int32_t* __restrict__ dsym, const int32_t* __restrict__ wave_p0,
                                                  const uint32_t* __restrict__ chan, EqTabs T) {
  __shared__ uint4 stage_all[kDfWaves][kDfUnits];
  __shared__ __attribute__((aligned(16))) uint32_t lut_all[256 * kDfLutCopies];   // copies of entry i at i * copies ..
  {
    uint32_t v[256 / kDfThreads];                      // (every load in flight, then the stores)
#pragma unroll
    for (int j = 0; j < 256 / kDfThreads; j++) v[j] = kDemapLut[threadIdx.x + j * kDfThreads];
#pragma unroll
    for (int j = 0; j < 256 / kDfThreads; j++)
#pragma unroll
      for (int c = 0; c < kDfLutCopies; c++) lut_all[(threadIdx.x + j * kDfThreads) * kDfLutCopies + c] = v[j];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint4* stage = stage_all[wv];
  const uint32_t* lut = lut_all + (lane & (kDfLutCopies - 1));
  const int total = dsym[npkts];
  const int nw = (total + 63) >> 6;
  const int wstep = gridDim.x * kDfWaves;
  int w = __builtin_amdgcn_readfirstlane(blockIdx.x * kDfWaves + wv);
  DfSym d;
  if (w < nw) {
    DfNext n;
    df_locate(w, lane, total, npkts, sym_off, vparams, soft_off, dsym, wave_p0, n);
    d = df_finish(n);
  }
  for (; w < nw; w += wstep) {
    s2 x[64];
    load_symbol(sym + (size_t)d.sidx * 16, x);
    const int wn = w + wstep;
    DfNext n;
    if (wn < nw) df_locate(wn, lane, total, npkts, sym_off, vparams, soft_off, dsym, wave_p0, n);
    // ---- compute
    const uint32_t* cp = EQ ? chan + (int64_t)d.p * 64 : nullptr;
    if (d.valid) {
      // the FFT (and EQ) for every lane at once, then the demapper of the lane's modulation:
      // with the FFT inside the per-modulation branches a wave whose symbols mix modulations
      // (config 5) ran it once per modulation present
      fft64_inplace(x);
      if constexpr (EQ) equalize_data_bins(x, [cp](int b) { return as_s2(cp[b]); }, d.k + 1, T);
      uint4* row = stage + kDfRow * lane;
      auto st = [row](int q, uint4 v) { row[q] = v; };
      auto lu = [lut](uint32_t i) { return lut[i * kDfLutCopies]; };
#if ZRX_DF_LUT_ONCE
      // the LUT once for every lane, then the packing of the lane's modulation: a wave whose
      // symbols mix modulations (config 5) no longer reads the LUT once per modulation present
      uint32_t lr[48], li[48];
      demap_lut_words(x, lu, lr, li);
      switch (d.mod) {
        case 0: demap_pack_st<0>(lr, li, st); break;
        case 1: demap_pack_st<1>(lr, li, st); break;
        case 2: demap_pack_st<2>(lr, li, st); break;
        default: demap_pack_st<3>(lr, li, st); break;
      }
#else
      switch (d.mod) {
        case 0: demap_deinterleave_st<0>(x, lu, st); break;
        case 1: demap_deinterleave_st<1>(x, lu, st); break;
        case 2: demap_deinterleave_st<2>(x, lu, st); break;
        default: demap_deinterleave_st<3>(x, lu, st); break;
      }
#endif
    }
    __builtin_amdgcn_wave_barrier();
    // ---- out: NU x 64 units, (s, q) = divmod(64j + lane, NU), NU = the wave's widest soft
    // row (3, 6, 12 or 18 units): a wave of BPSK / QPSK / 16-QAM symbols (mixed batches) runs
    // 3 / 6 / 12 store iterations, not 18
    // (lane0 is lane through an opaque move: the divmods are recomputed here each time
    // instead of being hoisted out of the loop as 54 live registers)
    int lane0;
    asm volatile("v_mov_b32 %0, %1" : "=v"(lane0) : "v"(lane));
    auto out = [&](auto nc) {
      constexpr int NU = decltype(nc)::value;
#pragma unroll
      for (int j = 0; j < NU; j++) {
        const int u = 64 * j + lane0;
        const int s = u / NU, q = u - NU * s;
        const uint32_t o = (uint32_t)__shfl((int)d.obase, s), nu = (uint32_t)__shfl((int)d.nu, s);
        const uint4 v = stage[kDfRow * s + q];
        if ((uint32_t)q < nu) soft[o + q] = v;
      }
    };
    if (__builtin_amdgcn_ballot_w64(d.nu > 12u)) out(std::integral_constant<int, 18>{});
    else if (__builtin_amdgcn_ballot_w64(d.nu > 6u)) out(std::integral_constant<int, 12>{});
    else if (__builtin_amdgcn_ballot_w64(d.nu > 3u)) out(std::integral_constant<int, 6>{});
    else out(std::integral_constant<int, 3>{});
    __builtin_amdgcn_wave_barrier();
    if (wn < nw) d = df_finish(n);
  }
}

// FFT >>> ChannelEqualization >>> PilotTrack (receiver.blk:66-69) with PilotTrack's full
// 64-bin output (bins 0 and 27..37 are zero, PilotTrack.blk:224-227); out has sym's layout.
// One wave per packet, lane = symbol.
__global__ __launch_bounds__(256) void k_ofdm_eq(const uint4* __restrict__ sym, const int64_t* __restrict__ sym_off,
                                                 const int32_t* __restrict__ nsym, int npkts,
                                                 const uint32_t* __restrict__ chan, EqTabs T, uint4* __restrict__ out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int p = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wv);
  if (p >= npkts) return;
  const uint32_t* cp = chan + (int64_t)p * 64;
  const int n = nsym[p];
  for (int k = lane; k < n; k += 64) {
    const int64_t so = (sym_off[p] + k) * 16;
    s2 x[64];
    load_symbol(sym + so, x);
    fft64_inplace(x);
    const s2 p1 = vmul_c16(x[bitrev6(43)], as_s2(cp[43]), 8), p2 = vmul_c16(x[bitrev6(57)], as_s2(cp[57]), 8);
    const s2 p3 = vmul_c16(x[bitrev6(7)], as_s2(cp[7]), 8), p4 = vmul_c16(x[bitrev6(21)], as_s2(cp[21]), 8);
    int avg, del;
    pilot_phase(p1, p2, p3, p4, k, T.atan, avg, del);
    uint32_t o[64];
#pragma unroll
    for (int b = 0; b < 64; b++) {
      if ((b >= 1 && b <= 26) || b >= 38)
        o[b] = as_u32(vmul_c16(vmul_c16(x[bitrev6(b)], as_s2(cp[b]), 8), rot_coeff(avg, del, b, T.rot), 15));
      else
        o[b] = 0u;
    }
    uint4* dst = out + so;
#pragma unroll
    for (int q = 0; q < 16; q++) dst[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
  }
}

// ------------------------------------------------------------------ descramble + CRC
// info[8p+4] = crc_ok, info[8p+7] = viterbi bits; payload gets len-4 descrambled bytes.
// One wave per packet, kCrcWaves packets per block.  The kernel is VALU-bound (8 waves a SIMD,
// ≈ 500 instructions a packet before this form), so the work per packet is what counts:
//  * Descrambler (Decode.blk:36-43, scramble.blk:28-44): the keystream of SERVICE state S is
//    one 127-periodic byte sequence read from phase 16*phase(S), so the payload is written
//    with coalesced dword stores (256 B per store instruction).  Dword i = decoded bytes
//    2+4i .. 5+4i: the upper neighbour word comes from lane + 1 by a wave_shl DPP move, the
//    keystream word from a table indexed by 32 x byte offset mod 127 (4 x 32 = 1 mod 127, so
//    consecutive lanes read consecutive words: no bank conflicts, no wrap test), bytes past the
//    payload are masked (one 64-bit shift, in the iterations that reach the payload's end).
//    The masked words also go to the wave's LDS copy (below).
//  * CRC-32 check (crc.blk:85-118, = zlib): by linearity the reference's all-ones-initialised
//    register is the zero-initialised one XOR kCrcOnes[n] (the all-ones value after n zero
//    bytes), and leading zero bytes leave a zero register unchanged, so the payload is
//    right-aligned in a 2048-byte frame and lane L takes bytes [32L, 32L+32) (slicing-by-4)
//    straight from the LDS copy — zeros before the payload, no keystream, no masks.  Each
//    lane's register is advanced past the 32*(63-L) bytes behind its chunk with two
//    nibble-sliced zero-byte tables of its own (((63-L) & 7) x 32 and ((63-L) >> 3) x 256
//    bytes: 16 lookups) and the wave XORs the 64 registers.
//  * LDS layouts, for bank conflicts (ds_read_b32: 32 banks per 32 lanes; b128: 64 banks per
//    16 lanes): the payload copy is indexed by v = i + 16 + u, u = (-c) & 7 for the chunk offset
//    c = (plen - 2048) >> 2, so every lane's chunk starts at a multiple of 8 (v 0..15 static
//    zeros, v 16..23 zeroed per packet before the payload lands) and is read by two ds_read_b128;
//    v sits at v ^ (((v >> 6) & 1) << 2), which puts 16 consecutive chunks on 16 distinct 4-bank
//    groups (unswizzled stride-8 words were 8-way conflicted).  The shift tables' rows are 144
//    words apart so odd and even rows use opposite bank halves.
constexpr int kCrcWaves = 8;
constexpr int kCrcGuard = 16;                         // static zero words (v) before a packet's copy
constexpr int kCrcRegion = 544;                       // per wave: v 0 .. 534 (16 + 7 + 512 words)
constexpr int kShfRow = 144;
__device__ __forceinline__ int crc_lds_pos(int v) { return v ^ (((v >> 6) & 1) << 2); }
__global__ __launch_bounds__(64 * kCrcWaves) void k_descramble_crc(const uint8_t* __restrict__ dec,
                                                                   const int32_t* __restrict__ dec_bits,
                                                                   int32_t* __restrict__ info, uint8_t* __restrict__ payload,
                                                                   int npkts) {
  __shared__ uint32_t s4[4][256];
  __shared__ uint32_t shf[16][kShfRow];               // [n]: n * 32 zero bytes, [8 + n]: n * 256
  __shared__ uint32_t scrw4[320];                     // keystream words: [j] = kScrW[4j mod 127]
  __shared__ uint8_t scrb[256];
  __shared__ uint8_t scrph[128];
  __shared__ __attribute__((aligned(16))) uint32_t pw_all[kCrcWaves][kCrcRegion];   // per wave: payload copy
  {                                                    // every table load in flight at once
    static_assert(64 * kCrcWaves == 512, "two words of each 1024-word table per thread");
    const int t = threadIdx.x;
    const uint32_t* S4 = &kCrcS4[0][0];
    const uint32_t* SL = &kCrcShiftLo[0][0];
    const uint32_t* SH = &kCrcShiftHi[0][0];
    const uint32_t a0 = S4[t], a1 = S4[t + 512], b0 = SL[t], b1 = SL[t + 512], c0 = SH[t], c1 = SH[t + 512];
    const uint32_t d2 = kScrW[(4 * t) % 127];
    const uint8_t e = kScrB2[min(t, 253)], f = kScrPhase[t & 127];
    (&s4[0][0])[t] = a0; (&s4[0][0])[t + 512] = a1;
    shf[t >> 7][t & 127] = b0; shf[4 + (t >> 7)][t & 127] = b1;
    shf[8 + (t >> 7)][t & 127] = c0; shf[12 + (t >> 7)][t & 127] = c1;
    if (t < 320) scrw4[t] = d2;
    if (t < 254) scrb[t] = e;
    if (t < 128) scrph[t] = f;
    if ((t & 63) < kCrcGuard) pw_all[t >> 6][t & 63] = 0u;   // (v < 64: position = v)
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // (packet values below: scalar)
  uint32_t* pw = pw_all[wv];                          // v at pw[crc_lds_pos(v)]
  // grid-stride over packets (one wave per packet at a time): the LDS tables above are
  // staged once per block, not once per 8 packets.  Decoded bytes are read and payload
  // dwords written by buffer ops on the packet's own slot: 32-bit lane offsets, and a word
  // outside the slot (load: 0) or past the payload (store: dropped) needs no branch.
  // Each packet's LENGTH is read one packet ahead (the first one before the tables are staged),
  // so its slot loads can stop at the decoded bytes the packet has: len + 2, plus the next
  // dword the descrambler aligns against (the slot is kDecStride = 2080 bytes; reading it all
  // fetched 1.42x the bytes a config-3 packet needs).
  int p = blockIdx.x * kCrcWaves + wv;
  int len_next = p < npkts ? info[8 * (int64_t)p + 2] : 0;
  for (; p < npkts; p += gridDim.x * kCrcWaves) {
    int32_t* in = info + 8 * (int64_t)p;
    const uint8_t* d = dec + (int64_t)p * kDecStride;
    const int len = len_next;
    const int pn = p + gridDim.x * kCrcWaves;
    if (pn < npkts) len_next = info[8 * (int64_t)pn + 2];
    const int nrec = min(kDecStride, (max(len, 0) + 2 + 4 + 3) & ~3);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)d, (short)0, nrec, 0x00020000);
    // payload: dword i = decoded bytes 2+4i .. 5+4i.  The lane's dwords i = lane + 64k
    // (k < 8: plen <= 2044) are loaded with the header fields, before any of them is looked at
    // (a packet that turns out to have no payload wastes them; loads past nrec read 0 and
    // fetch nothing).
    uint32_t wv9[9];
#pragma unroll
    for (int k = 0; k < 9; k++) wv9[k] = __builtin_amdgcn_raw_buffer_load_b32(rd, 4 * (lane + 64 * k), 0, 0);
    const int status = in[5];
    const int bits = dec_bits[p];
    if (lane == 0) in[7] = bits;
    if (status != 0 || bits < (len + 2) * 8 || len < 4) {
      if (lane == 0) in[4] = 0;
      continue;
    }
    const int plen = len - 4;
    // the received CRC: decoded bytes 2 + plen .. 5 + plen (scalar loads, used at the end)
    const uint32_t* dw = (const uint32_t*)d;
    const int tb = (2 + plen) >> 2;
    const uint32_t t0 = dw[tb], t1 = dw[tb + 1];
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc((void*)(payload + (int64_t)p * kPayloadStride),
                                                                         (short)0, (plen + 3) & ~3, 0x00020000);
    // SERVICE bits 9..15 = scrambler state (decoded byte 1: lane 0's first word)
    const uint32_t S = ((uint32_t)__builtin_amdgcn_readfirstlane((int)wv9[0]) >> 9) & 0x7Fu;
    const uint32_t ksm = S == 0 ? 0u : 0xFFFFFFFFu;   // state 0 never leaves 0: zero keystream
    const int n0 = (16 * (int)scrph[S]) % 127;
    // keystream word of dword i = lane + 64k: kScrW[(n0 + 4i) mod 127] = scrw4[j] for j = 32 (n0 + 4i)
    // mod 127 = (32 n0 mod 127) + lane + (64k mod 127): consecutive lanes, consecutive words
    const uint32_t* ks = scrw4 + (4 * (int)scrph[S]) % 127 + lane;   // (32 n0 = 512 phase = 4 phase)
    const int c = (plen - 2048) >> 2;                  // payload word of lane 0's CRC chunk (floor)
    const int u = (-c) & 7;
    if (lane < 8) pw[16 + lane] = 0u;                  // v 16 .. 15 + u: zero (the rest: overwritten)
    const int v0 = lane + kCrcGuard + u;               // v of dword lane + 64k: v0 + 64k
    const int pe = crc_lds_pos(v0), po = pe ^ 4;       // its position, k even / odd
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int i = lane + 64 * k;
      // dword i + 1: lane + 1's word k (wave_shl:1), lane 63's from lane 0's word k + 1
      const uint32_t up = (uint32_t)__builtin_amdgcn_readfirstlane((int)wv9[k + 1]);
      const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp((int)up, (int)wv9[k], 0x130, 0xF, 0xF, false);
      uint32_t v = __builtin_amdgcn_alignbyte(nx, wv9[k], 2) ^ (ks[(k >> 1) + 64 * (k & 1)] & ksm);
      if (4 * (64 * k + 64) > plen)                    // (wave-uniform) bytes past the payload := 0
        v &= (uint32_t)(0xFFFFFFFFull >> (32 - 8 * min(max(plen - 4 * i, 0), 4)));
      __builtin_amdgcn_raw_buffer_store_b32(v, rp, 4 * i, 0, 0);   // (past the payload: dropped)
      pw[(k & 1 ? po : pe) + 64 * k] = v;
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t crc;
    if (plen >= 4) {
      // lane L's chunk: payload words 8L + c .. 8L + c + 8 at v = 8L + 16 + (c + u), a multiple
      // of 8; a chunk wholly before v = 0 is all zeros, read from v 0..7.  Word 8 is word 0 of
      // lane L + 1's chunk (lane 63: v = 528 + c + u, read by every lane as one broadcast).
      const int vl = max(8 * lane + kCrcGuard + c + u, 0);
      const int sh = plen & 3;                         // (byte offset of every lane's chunk)
      const int p0 = crc_lds_pos(vl);
      const uint4 lo = *(const uint4*)(pw + p0), hi = *(const uint4*)(pw + (p0 ^ 4));
      const uint32_t last = pw[crc_lds_pos(528 + c + u)];
      uint32_t w[9] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w, 0u};
      w[8] = (uint32_t)__builtin_amdgcn_update_dpp((int)last, (int)lo.x, 0x130, 0xF, 0xF, false);
      uint32_t r = 0;
#pragma unroll
      for (int j = 0; j < 8; j++) {
        r ^= __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
        r = s4[3][r & 0xFFu] ^ s4[2][(r >> 8) & 0xFFu] ^ s4[1][(r >> 16) & 0xFFu] ^ s4[0][r >> 24];
      }
      // advance past the 63 - lane 32-byte chunks behind this one: (63 - lane) & 7 chunks,
      // then (63 - lane) >> 3 times 256 bytes (the lane's two tables; entry 0 is the identity)
      const uint32_t adv = 63u - (uint32_t)lane;
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const uint32_t* tb2 = shf[k ? 8u + (adv >> 3) : (adv & 7u)];   // (rows kShfRow apart)
        uint32_t t = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) t ^= tb2[j * 16 + ((r >> (4 * j)) & 15u)];
        r = t;
      }
      crc = ~(wave_xor_u32(r) ^ kCrcOnes[plen]);
    } else {                                           // < 4 payload bytes: the plain register
      crc = 0xFFFFFFFFu;
      for (int q = 0; q < plen; q++)
        crc = s4[0][(crc ^ ((uint32_t)d[2 + q] ^ (scrb[n0 + q] & ksm))) & 0xFFu] ^ (crc >> 8);
      crc = ~crc;
    }
    if (lane == 0) {
      const uint32_t rx = __builtin_amdgcn_alignbyte(t1, t0, (2 + plen) & 3) ^ (scrw4[(32 * (n0 + plen)) % 127] & ksm);
      in[4] = crc == rx ? 1 : 0;
    }
    __builtin_amdgcn_wave_barrier();                   // (this packet's LDS reads before the next one's writes)
  }
}

}  // namespace zrx
