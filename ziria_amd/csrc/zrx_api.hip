// Host side of libziria_rx.so: the device API (Part 3) and the batched externals (Part 2) of
// include/ziria_rx.h.
//
// Everything here computes in the HIP kernels of zrx_kernels.hip on a gfx950 device; this
// file only validates arguments, stages buffers and launches.  Without a usable GPU every
// entry point fails loudly (message on stderr + error code); there is no CPU fallback.  The
// per-call externals (Part 1) are the host path of zrx_host.cpp, by design.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <array>
#include <cmath>
#include <mutex>
#include <vector>

#define ZRX_C_LINKAGE_EXTERNALS
#include "../../include/ziria_rx.h"
#include "zrx_internal.h"
#include "zrx_kernels.hip"
#include "zrx_hostio.hpp"
#include "zrx_shard.hpp"

using namespace zrx;

#define ZRX_CHECK(call)                                                                   \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess) {                                                               \
      std::fprintf(stderr, "ziria_rx: HIP error %s at %s:%d\n", hipGetErrorString(e_),   \
                   __FILE__, __LINE__);                                                   \
      return ZRX_EHIP;                                                                    \
    }                                                                                     \
  } while (0)

struct zrx_ctx {
  int device = 0;
  int ncu = 256;                  // compute units (k_pkt_plan: segment length, block placement)
  int crc_blocks = 1024;          // k_descramble_crc grid cap (blocks of kCrcWaves packets)
  int df_blocks = 512, df_blocks_eq = 512;   // k_data_fft grid: the blocks resident at once (no tail round)
#ifdef ZRX_EXPERIMENTS
  // A/B builds only (scripts/build_variant.sh): environment knobs that select other kernels
  int v3dbg = 0;                  // ZRX_V3DBG: k_viterbi3 timing-experiment variants (wrong output)
#endif
  hipStream_t stream = nullptr;
  bool owns_stream = false;       // a shard context of the batched externals: its own stream
  bool timing = false;
  // one set of 6 events per timed zrx_rx_dev launch since zrx_enable_timing (averaged by
  // zrx_get_timing), so stages are timed live inside a run of back-to-back launches
  std::vector<std::array<hipEvent_t, 6>> evsets;
  size_t nrec = 0;
  // rx-chain workspace (zrx_reserve)
  int cap_pkts = 0, cap_nsym = 0;
  int64_t soft_stride = 0;
  uint32_t* sig_soft = nullptr;   // 48 B per packet
  int32_t* vparams = nullptr;     // 4 int32 per packet
  uint8_t* soft = nullptr;        // soft_stride B per packet
  int64_t* soft_off = nullptr;    // per packet, packed by soft_len (k_pkt_plan)
  int32_t* dsym = nullptr;        // data-symbol prefix per packet, npkts + 1 (k_pkt_plan)
  int32_t* wave_p0 = nullptr;     // first packet of each k_data_fft wave (k_pkt_plan)
  uint8_t* dec = nullptr;         // kDecStride B per packet
  int64_t* dec_off = nullptr;     // p * kDecStride
  int32_t* dec_bits = nullptr;
  // k_viterbi3's row table (k_pkt_plan): segments of the batch's frames in decode order
  int2* rows = nullptr;           // {packet, k | nseg << 8}, at most rows_cap
  int32_t* nrows = nullptr;       // rows planned for the current launch
  uint8_t* segs = nullptr;        // segments per packet
  int32_t* order = nullptr;       // k_pkt_plan scratch: packets in row order
  uint2* dumps = nullptr;         // seam metric dumps, v3::seam_index
  PlanScanRec* scan_rec = nullptr; // k_pkt_scan's per-block records (ceil(npkts / 4096) + 1)
  uint32_t* scan_ctr = nullptr;   // its finished-block counter (reset by the last block)
  uint32_t scan_epoch = 0;        // its ready mark, one per launch (never 0: records start zeroed)
  int64_t rows_cap = 0;
  bool use_order = true;          // ZRX_ORDER=0 (experiment builds) turns the plan off
  // The workspace is shared by every launch of this context: a launch on a different stream
  // than the previous one first waits for the previous launch's work (ws_free).
  hipEvent_t ws_free = nullptr;
  hipStream_t ws_stream = nullptr;
  bool ws_pending = false;
  // ChannelEqualization / PilotTrack trig tables (built on first use)
  uint32_t* eq_rot = nullptr;     // 65536 x (cos, -sin) complex16
  int16_t* eq_atan = nullptr;     // 256 x 256 atan2x_lut
  // RX front end (zrx_rx_stream_dev): STS pattern and per-capture staging, grown on demand
  uint32_t* fe_pattern = nullptr; // 16 x 16 complex16
  int fe_cap = 0, fe_sym = 0;     // captures x symbols per capture the staging holds
  uint32_t* fe_syms = nullptr;
  int64_t* fe_sym_off = nullptr;
  int32_t* fe_nsym = nullptr;
  uint32_t* fe_chan = nullptr;
  uint32_t* tx_preamble = nullptr; // 640 complex16 (TX, createPreamble.blk)
  // FFTSafe<N> plans of every __ext_sora_fft size (zrx_fftn.hpp), built on first use
  FftPlan* fft_plans = nullptr;
  uint32_t* fft_tw = nullptr;
  uint16_t* fft_pos = nullptr;
  void* small = nullptr;          // device buffers of the batched externals' host arrays
  size_t small_cap = 0;
  zrx_io::HostIO* hio = nullptr;  // their copy streams and pinned slots (zrx_hostio.hpp)
  hipStream_t side = nullptr;     // k_pkt_rows beside k_data_fft (rx chain, mixed batches)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  int32_t* mixed_hint = nullptr;  // pinned, mapped: 1 when the last planned batch was mixed
  int32_t* mixed_hint_dev = nullptr;
  // zrx_pipeline_link: the context taking the other half of a stream of batches
  zrx_ctx* peer = nullptr;
  int link_mode = 0;
  hipEvent_t ev_vit_done = nullptr, ev_chain_done = nullptr;   // recorded every chain while linked
  // link mode 4: the chain's head (SIGNAL .. k_data_fft) on a low-priority stream of its own,
  // forked from and joined back into the caller's stream
  hipStream_t lo = nullptr;
  hipEvent_t ev_lo_fork = nullptr, ev_lo_join = nullptr;
};

static int check_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device) {
    std::fprintf(stderr, "ziria_rx: no HIP device %d available (this engine has no CPU path)\n", device);
    return ZRX_ENODEV;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return ZRX_ENODEV;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    std::fprintf(stderr, "ziria_rx: device %d is %s, this build targets gfx950\n", device, prop.gcnArchName);
    return ZRX_ENODEV;
  }
  return ZRX_OK;
}

static void free_ws(zrx_ctx* c) {
  for (void* p : {(void*)c->sig_soft, (void*)c->vparams, (void*)c->soft, (void*)c->soft_off, (void*)c->dsym,
                  (void*)c->wave_p0, (void*)c->dec, (void*)c->dec_off, (void*)c->dec_bits, (void*)c->rows,
                  (void*)c->nrows, (void*)c->segs, (void*)c->dumps, (void*)c->order, (void*)c->scan_rec,
                  (void*)c->scan_ctr})
    (void)hipFree(p);
  c->scan_rec = nullptr; c->scan_ctr = nullptr;
  c->sig_soft = nullptr; c->vparams = nullptr; c->soft = nullptr; c->soft_off = nullptr;
  c->dsym = nullptr; c->wave_p0 = nullptr; c->dec = nullptr; c->dec_off = nullptr; c->dec_bits = nullptr;
  c->rows = nullptr; c->nrows = nullptr; c->segs = nullptr; c->dumps = nullptr; c->order = nullptr; c->rows_cap = 0;
  c->cap_pkts = c->cap_nsym = 0;
}

__global__ void k_fill_offsets(int64_t* off, int n, int64_t stride) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) off[i] = (int64_t)i * stride;
}

static inline int blocks(int64_t n, int per) { return (int)((n + per - 1) / per); }
#ifndef ZRX_SIGFFT_LANES
#define ZRX_SIGFFT_LANES 64
#endif
constexpr int kSigFftLanes = ZRX_SIGFFT_LANES;
static_assert(kSigFftLanes % 64 == 0, "k_signal_fft stages its LUT with 64-thread strides");

// Trig tables of ChannelEqualization / PilotTrack: the reference LUTs (csrc/intalglutx.h:23,
// :3667, :7351) in closed form, with pi written as 3.141593 as their generator did:
// sinx/cosx[r] = rint(32767 sin/cos(2 r pi' / 65536)), atan2x[(u8)y][(u8)x] =
// trunc(atan2(y, x) / pi' * 32768).  Checked entry by entry against the reference tables.
static void make_trig_tables(int16_t* sinv, int16_t* cosv, int16_t* atanv) {
  const double pi = 3.141593;
  for (int r = 0; r < 65536; r++) {
    sinv[r] = (int16_t)std::nearbyint(32767.0 * std::sin((double)r * 2.0 * pi / 65536.0));
    cosv[r] = (int16_t)std::nearbyint(32767.0 * std::cos((double)r * 2.0 * pi / 65536.0));
  }
  for (int i = 0; i < 256; i++)
    for (int j = 0; j < 256; j++)
      atanv[(i << 8) | j] = (int16_t)std::trunc(std::atan2((double)(int8_t)i, (double)(int8_t)j) / pi * 32768.0);
}

// ---- RX front end host tables -------------------------------------------------------
// IFFT<64> (csrc/ifft_r4difx.hpp:56-250) for createSTSinTime (cca_tufv.blk:50-77); host
// code, run once per context.  Saturating int16 (adds/subs), XOR-as-negate, conj_mul_shiftx
// (csrc/sora_ext_lib_fft.hpp:68-94) with 32-bit madd wrap, 6-bit bit-reversed output.
namespace hostfft {
struct c16 { int16_t re, im; };
static inline int16_t sat(int32_t x) { return (int16_t)std::min(32767, std::max(-32768, x)); }
static inline int16_t inv(int16_t x) { return (int16_t)~x; }
static inline c16 add(c16 a, c16 b) { return {sat(a.re + b.re), sat(a.im + b.im)}; }
static inline c16 sub(c16 a, c16 b) { return {sat(a.re - b.re), sat(a.im - b.im)}; }
static inline c16 shr2(c16 a) { return {(int16_t)(a.re >> 2), (int16_t)(a.im >> 2)}; }
static inline c16 cmul(c16 a, int16_t br, int16_t bi) {
  const int32_t re = (int32_t)((uint32_t)(a.re * br) + (uint32_t)(a.im * bi));
  const int32_t im = (int32_t)((uint32_t)(a.im * br) + (uint32_t)(inv(a.re) * bi));
  return {(int16_t)(re >> 15), (int16_t)(im >> 15)};
}
static void stage(c16* x, int N) {
  const int16_t* t1 = N == 64 ? kTw64_1 : kTw16_1;
  const int16_t* t2 = N == 64 ? kTw64_2 : kTw16_2;
  const int16_t* t3 = N == 64 ? kTw64_3 : kTw16_3;
  for (int n = 0; n < N / 4; n++) {
    const c16 a = shr2(x[n]), b = shr2(x[n + N / 4]), c = shr2(x[n + N / 2]), d = shr2(x[n + 3 * N / 4]);
    const c16 ac = add(a, c), bd = add(b, d), a_c = sub(a, c), b_d = sub(b, d);
    x[n] = add(ac, bd);
    x[n + N / 4] = cmul(sub(ac, bd), t2[2 * n], t2[2 * n + 1]);
    const c16 jb = {inv(b_d.im), b_d.re};
    x[n + N / 2] = cmul(add(a_c, jb), t1[2 * n], t1[2 * n + 1]);
    x[n + 3 * N / 4] = cmul(sub(a_c, jb), t3[2 * n], t3[2 * n + 1]);
  }
}
static void four(c16* x) {      // IFFTSSEEx<4> (:114-150)
  const c16 y0 = shr2(x[0]), y1 = shr2(x[1]), y2 = shr2(x[2]), y3 = shr2(x[3]);
  const c16 A = add(y0, y2), B = add(y1, y3);
  const c16 C = add(y0, {inv(y2.re), inv(y2.im)}), D = add(y1, {inv(y3.re), inv(y3.im)});
  const c16 jD = {inv(D.im), D.re};
  x[0] = add(A, B);
  x[1] = add({inv(B.re), inv(B.im)}, A);
  x[2] = add(C, jD);
  x[3] = add({inv(jD.re), inv(jD.im)}, C);
}
static void eight(c16* x) {     // IFFTSSEEx<8> (:152-228)
  c16 sm[4], e[4];
  for (int k = 0; k < 4; k++) {
    const c16 a = {(int16_t)(x[k].re >> 3), (int16_t)(x[k].im >> 3)}, b = {(int16_t)(x[k + 4].re >> 3), (int16_t)(x[k + 4].im >> 3)};
    sm[k] = add(a, b);
    e[k] = sub(a, b);
  }
  const c16 A = add(sm[0], sm[2]), B = add(sm[1], sm[3]);
  const c16 C = add({inv(sm[2].re), inv(sm[2].im)}, sm[0]), D = add({inv(sm[3].re), inv(sm[3].im)}, sm[1]);
  const c16 jD = {inv(D.im), D.re};
  c16 o[8];
  o[0] = add(A, B); o[1] = add({inv(B.re), inv(B.im)}, A);
  o[2] = add(C, jD); o[3] = add({inv(jD.re), inv(jD.im)}, C);
  const c16 je2 = {inv(e[2].im), e[2].re}, je3 = {inv(e[3].im), e[3].re};
  const c16 u0 = cmul(add(e[0], je2), 32767, 0), u1 = cmul(add(e[1], je3), 23169, -23169);
  const c16 u2 = cmul(add({inv(je2.re), inv(je2.im)}, e[0]), 32767, 0);
  const c16 u3 = cmul(add({inv(je3.re), inv(je3.im)}, e[1]), -23169, -23169);
  o[4] = add(u0, u1); o[5] = add({inv(u1.re), inv(u1.im)}, u0);
  o[6] = add(u2, u3); o[7] = add({inv(u3.re), inv(u3.im)}, u2);
  std::memcpy(x, o, sizeof(o));
}
static void stage_n(c16* x, int N, const int16_t* t1, const int16_t* t2, const int16_t* t3) {
  for (int n = 0; n < N / 4; n++) {
    const c16 a = shr2(x[n]), b = shr2(x[n + N / 4]), c = shr2(x[n + N / 2]), d = shr2(x[n + 3 * N / 4]);
    const c16 ac = add(a, c), bd = add(b, d), a_c = sub(a, c), b_d = sub(b, d);
    x[n] = add(ac, bd);
    x[n + N / 4] = cmul(sub(ac, bd), t2[2 * n], t2[2 * n + 1]);
    const c16 jb = {inv(b_d.im), b_d.re};
    x[n + N / 2] = cmul(add(a_c, jb), t1[2 * n], t1[2 * n + 1]);
    x[n + 3 * N / 4] = cmul(sub(a_c, jb), t3[2 * n], t3[2 * n + 1]);
  }
}
static void ifft128(const c16* in, c16* out) {
  c16 x[128];
  std::memcpy(x, in, sizeof(x));
  stage_n(x, 128, kTw128_1, kTw128_2, kTw128_3);
  for (int q = 0; q < 4; q++) {
    stage_n(x + 32 * q, 32, kTw32_1, kTw32_2, kTw32_3);
    for (int r = 0; r < 4; r++) eight(x + 32 * q + 8 * r);
  }
  for (int i = 0; i < 128; i++) out[i] = x[tx::bitrev7(i)];
}
static void ifft64(const c16* in, c16* out) {
  c16 x[64];
  std::memcpy(x, in, sizeof(x));
  stage(x, 64);
  for (int q = 0; q < 4; q++) {
    stage(x + 16 * q, 16);
    for (int r = 0; r < 4; r++) four(x + 16 * q + 4 * r);
  }
  for (int i = 0; i < 64; i++) out[i] = x[bitrev6(i)];
}
}  // namespace hostfft

// InitCorrPattern (cca_tufv.blk:80-98): pattern[16 i + j] = (sts_time[i + j] >> 7)
static void make_cca_pattern(uint32_t* pattern) {
  const int16_t m = (int16_t)(10720.0 * 1.472);      // int16(double(bpsk_mod_11a) * 1.472)
  hostfft::c16 sts[64] = {}, t[64];
  const int pos[12] = {4, 8, 12, 16, 20, 24, 40, 44, 48, 52, 56, 60};
  const int sgn[12] = {-1, -1, 1, 1, 1, 1, 1, -1, 1, -1, -1, 1};
  for (int i = 0; i < 12; i++) sts[pos[i]] = {(int16_t)(sgn[i] * m), (int16_t)(sgn[i] * m)};
  hostfft::ifft64(sts, t);
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 16; j++) {
      const hostfft::c16 v = t[i + j];
      pattern[16 * i + j] = (uint32_t)(uint16_t)(v.re >> 7) | ((uint32_t)(uint16_t)(v.im >> 7) << 16);
    }
}

// createSTSinTime / createLTSinTime at 40 MHz (transmitter/createPreamble.blk:38-117)
static void make_tx_preamble(uint32_t* out640) {
  const int16_t sm = (int16_t)(10720.0 * 1.472), lm = 10720;
  hostfft::c16 f[128] = {}, t[128];
  const int sp[12] = {4, 8, 12, 16, 20, 24, 104, 108, 112, 116, 120, 124};
  const int ss[12] = {-1, -1, 1, 1, 1, 1, 1, -1, 1, -1, -1, 1};
  for (int i = 0; i < 12; i++) f[sp[i]] = {(int16_t)(ss[i] * sm), (int16_t)(ss[i] * sm)};
  hostfft::ifft128(f, t);
  auto w = [](hostfft::c16 v) { return (uint32_t)(uint16_t)v.re | ((uint32_t)(uint16_t)v.im << 16); };
  for (int i = 0; i < 320; i++) out640[i] = w(t[i < 256 ? i & 127 : i - 256]);
  hostfft::c16 g[128] = {};
  for (int i = 1; i <= 26; i++) g[i].re = ((kLts11aBits >> i) & 1ull) ? lm : (int16_t)-lm;
  for (int i = 38; i < 64; i++) g[i + 64].re = ((kLts11aBits >> i) & 1ull) ? lm : (int16_t)-lm;
  hostfft::ifft128(g, t);
  uint32_t* l = out640 + 320;
  for (int i = 0; i < 128; i++) l[64 + i] = l[192 + i] = w(t[i]);
  for (int i = 0; i < 64; i++) l[i] = l[256 + i];
}

// amp values where log2(1000 / sqrt(amp)) is an exact k + 0.5 (amp = 10^6 / 2^(2k+1)):
// their rounding follows this host libm, like the reference's round_int32(log2(...)).
static fe::AgcTies make_agc_ties() {
  fe::AgcTies t;
  for (int i = 0; i < 8; i++) {
    const int k = 2 - i;                              // k = 2 .. -5
    const double amp = 1e6 / std::ldexp(1.0, 2 * k + 1);
    t.amp[i] = (int32_t)amp;
    const double d = std::log(1000.0 / std::sqrt((double)t.amp[i])) / std::log(2.0);
    t.agc[i] = (int32_t)((d > 0) ? (d + 0.5) : (d - 0.5));
  }
  return t;
}

static int ensure_eq_tables(zrx_ctx* c) {
  if (c->eq_rot) return ZRX_OK;
  std::vector<int16_t> sv(65536), cv(65536), av(65536);
  make_trig_tables(sv.data(), cv.data(), av.data());
  std::vector<uint32_t> rot(65536);
  for (int r = 0; r < 65536; r++)     // build_coeff (PilotTrack.blk:28-50): (cos th, -sin th)
    rot[r] = (uint32_t)(uint16_t)cv[r] | ((uint32_t)(uint16_t)(int16_t)(-sv[r]) << 16);
  zrx_shard::DeviceGuard dg(c->device);   // (the caller's device is restored on return)
  ZRX_CHECK(hipMalloc(&c->eq_rot, 65536 * 4));
  ZRX_CHECK(hipMalloc(&c->eq_atan, 65536 * 2));
  ZRX_CHECK(hipMemcpy(c->eq_rot, rot.data(), 65536 * 4, hipMemcpyHostToDevice));
  ZRX_CHECK(hipMemcpy(c->eq_atan, av.data(), 65536 * 2, hipMemcpyHostToDevice));
  return ZRX_OK;
}

static bool order_fits(const zrx_ctx* c, int npkts) {
  return c->use_order && c->rows && npkts <= c->cap_pkts;
}

// Every launch function starts here: a launch on a different stream than the previous one
// waits for the previous launch's work on the shared workspace to finish.
static int ws_acquire(zrx_ctx* c) {
  // (stream-to-stream on one device: no system-scope fence; 0.1-0.7 % a step in A/B.  Recording
  // it only when a launch changes streams was 50 % slower with two linked engines.)
  if (!c->ws_free)
    ZRX_CHECK(hipEventCreateWithFlags(&c->ws_free, hipEventDisableTiming | hipEventDisableSystemFence));
  if (c->ws_pending && c->ws_stream != c->stream) ZRX_CHECK(hipStreamWaitEvent(c->stream, c->ws_free, 0));
  return ZRX_OK;
}
static int ws_release(zrx_ctx* c) {
  ZRX_CHECK(hipEventRecord(c->ws_free, c->stream));
  c->ws_stream = c->stream;
  c->ws_pending = true;
  return ZRX_OK;
}

// Rows a plan of npkts packets can have: sum of ceil(cols / L') <= total / L' + npkts with
// L' = L x kSegMixNum / 8 (mixed) or 9/8 L (uniform), total / L <= 64 ncu (k_pkt_plan), and
// at most kMaxSeg per packet.
static int64_t plan_rows_max(const zrx_ctx* c, int npkts) {
  // (+ 1/256 + 64: L x kSegMixNum / 8 rounds down, which can add a few rows over the ratio)
  // (a uniform batch is cut at 9/8 L, a mixed one at kSegMixNum / 8 L: the grid covers both)
  const int64_t r = 64 * 8 * (int64_t)c->ncu / std::min<int64_t>(v3::kSegMixNum, 8);
  return std::min<int64_t>((int64_t)npkts + r + r / 256 + 64, (int64_t)npkts * v3::kMaxSeg);
}

// planned: the caller already ran k_pkt_plan for this batch (rx chain)
static void launch_viterbi(zrx_ctx* c, const uint8_t* soft, const int64_t* soft_off, const int32_t* params,
                           int npkts, uint8_t* out, const int64_t* out_off, int32_t* out_bits,
                           bool planned = false) {
  // rows of a k_viterbi3 wave should share a rate and length, and long frames are cut into
  // segments when the batch is too small to fill the GPU: plan the batch first when the
  // workspace has room for it (zrx_reserve); otherwise one row per packet in batch order
  // (still exact)
  const bool plan = order_fits(c, npkts);
  if (plan && !planned)
    k_pkt_plan<<<1, 1024, 0, c->stream>>>(params, npkts, nullptr, nullptr, nullptr, c->rows, c->nrows, c->segs, c->order,
                                          out_bits, c->ncu, (int)plan_rows_max(c, npkts), 0, nullptr);
  const dim3 b(256);
  const dim3 g(blocks(plan ? plan_rows_max(c, npkts) : npkts, v3::kRows));
  const int2* rows = plan ? c->rows : nullptr;
  int32_t* nrows = plan ? c->nrows : nullptr;
#ifdef ZRX_EXPERIMENTS
  switch (c->v3dbg) {   // timing experiments (ZRX_V3DBG); 0 is the product kernel
#define ZRX_V3(D) case D: k_viterbi3<D><<<g, b, 0, c->stream>>>(soft, soft_off, params, npkts, out, out_off, out_bits, rows, nrows, nullptr, c->dumps); return;
    ZRX_V3(1) ZRX_V3(2) ZRX_V3(4) ZRX_V3(8) ZRX_V3(16) ZRX_V3(64) ZRX_V3(1024) ZRX_V3(1032) ZRX_V3(2048)
#undef ZRX_V3
    default: break;
  }
#endif
  k_viterbi3<0><<<g, b, 0, c->stream>>>(soft, soft_off, params, npkts, out, out_off, out_bits, rows, nrows, nullptr,
                                        c->dumps);
  // the seam pass: packets whose segments disagree at a seam are re-decoded from there
  // (normally none; a block-stride grid of at most 2 blocks per CU)
  if (plan)
    k_viterbi3<0, true><<<std::min(blocks(npkts, v3::kRows), 2 * c->ncu), b, 0, c->stream>>>(
        soft, soft_off, params, npkts, out, out_off, out_bits, nullptr, c->nrows, c->segs, c->dumps);
}

// ---- FFTSafe<N> plans (zrx_fftplan.hpp), uploaded once per context --------------------
static int fftn_plans(zrx_ctx* c) {
  if (c->fft_plans) return ZRX_OK;
  const FftPlans R = fftn_build_plans();
  const std::vector<FftPlan>& plans = R.plans;
  const std::vector<uint32_t>& tw = R.tw;
  const std::vector<uint16_t>& pos = R.pos;
  zrx_shard::DeviceGuard dg(c->device);   // (the caller's device is restored on return)
  ZRX_CHECK(hipMalloc(&c->fft_plans, sizeof(FftPlan) * kFftSizes));
  ZRX_CHECK(hipMalloc(&c->fft_tw, tw.size() * 4));
  ZRX_CHECK(hipMalloc(&c->fft_pos, pos.size() * 2));
  ZRX_CHECK(hipMemcpy(c->fft_plans, plans.data(), sizeof(FftPlan) * kFftSizes, hipMemcpyHostToDevice));
  ZRX_CHECK(hipMemcpy(c->fft_tw, tw.data(), tw.size() * 4, hipMemcpyHostToDevice));
  ZRX_CHECK(hipMemcpy(c->fft_pos, pos.data(), pos.size() * 2, hipMemcpyHostToDevice));
  return ZRX_OK;
}
// count transforms of nfft points on the context's stream (nfft supported, plans built)
static void launch_fft(zrx_ctx* c, int nfft, const void* d_in, void* d_out, int64_t count) {
  if (nfft == 64) {
    k_fft64<<<blocks(count, 256), 256, 0, c->stream>>>((const uint4*)d_in, (uint4*)d_out, count);
    return;
  }
  const int g = (int)std::min<int64_t>(count, 8 * (int64_t)c->ncu);
  k_fft_n<<<g, 256, 0, c->stream>>>((const uint32_t*)d_in, (uint32_t*)d_out, count, c->fft_plans + fftn_index(nfft),
                                     c->fft_tw, c->fft_pos);
}

extern "C" {

const char* zrx_version(void) { return "ziria_rx 0.1 (gfx950)"; }

int zrx_create(zrx_ctx** out, int device, void* stream) {
  if (!out) return ZRX_EINVAL;
  *out = nullptr;
  int rc = check_device(device);
  if (rc) return rc;
  zrx_shard::DeviceGuard dg(device);
  zrx_ctx* c = new zrx_ctx();
  c->device = device;
  ZRX_CHECK(hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, device));
  c->stream = (hipStream_t)stream;
  // k_data_fft loops its waves over the batch: launch exactly the blocks that are resident at
  // once (occupancy from its VGPRs and LDS), so no second round of blocks runs alone at the end
  int occ = 0;
  ZRX_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_data_fft<false>, kDfThreads, 0));
  c->df_blocks = std::max(1, occ) * c->ncu;
  ZRX_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_data_fft<true>, kDfThreads, 0));
  c->df_blocks_eq = std::max(1, occ) * c->ncu;
#ifdef ZRX_EXPERIMENTS
  if (const char* v = std::getenv("ZRX_V3DBG")) c->v3dbg = std::atoi(v);
  if (const char* v = std::getenv("ZRX_ORDER")) c->use_order = std::atoi(v) != 0;
  if (const char* v = std::getenv("ZRX_CRCBLOCKS")) c->crc_blocks = std::atoi(v);
  std::fprintf(stderr, "ziria_rx: EXPERIMENT build (v3dbg %d, order %d, crc_blocks %d)\n", c->v3dbg, (int)c->use_order,
               c->crc_blocks);
#else
  static bool warned = false;
  for (const char* k : {"ZRX_V3DBG", "ZRX_ORDER", "ZRX_CRCBLOCKS"})
    if (std::getenv(k) && !warned) {
      std::fprintf(stderr, "ziria_rx: %s is an experiment-build knob (scripts/build_variant.sh); ignored by this "
                           "product build\n", k);
      warned = true;
    }
#endif
  *out = c;
  return ZRX_OK;
}

int zrx_destroy(zrx_ctx* c) {
  if (!c) return ZRX_OK;
  zrx_shard::DeviceGuard dg(c->device);
  free_ws(c);
  (void)hipFree(c->eq_rot);
  (void)hipFree(c->eq_atan);
  for (void* p : {(void*)c->fe_pattern, (void*)c->fe_syms, (void*)c->fe_sym_off, (void*)c->fe_nsym, (void*)c->fe_chan,
                  (void*)c->tx_preamble})
    (void)hipFree(p);
  for (void* p : {(void*)c->fft_plans, (void*)c->fft_tw, (void*)c->fft_pos}) (void)hipFree(p);
  (void)hipFree(c->small);
  delete c->hio;
  if (c->mixed_hint) (void)hipHostFree(c->mixed_hint);
  for (auto& set : c->evsets)
    for (auto& e : set) (void)hipEventDestroy(e);
  if (c->ws_free) (void)hipEventDestroy(c->ws_free);
  if (c->peer) { c->peer->peer = nullptr; c->peer->link_mode = 0; }
  if (c->ev_vit_done) (void)hipEventDestroy(c->ev_vit_done);
  if (c->ev_chain_done) (void)hipEventDestroy(c->ev_chain_done);
  if (c->lo) {
    (void)hipStreamDestroy(c->lo);
    (void)hipEventDestroy(c->ev_lo_fork);
    (void)hipEventDestroy(c->ev_lo_join);
  }
  if (c->side) {
    (void)hipStreamDestroy(c->side);
    (void)hipEventDestroy(c->ev_fork);
    (void)hipEventDestroy(c->ev_join);
  }
  if (c->owns_stream && c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return ZRX_OK;
}

int zrx_set_stream(zrx_ctx* c, void* stream) {
  if (!c) return ZRX_EINVAL;
  c->stream = (hipStream_t)stream;
  return ZRX_OK;
}

int zrx_pipeline_link(zrx_ctx* a, zrx_ctx* b, int mode) {
  if (!a || !b || a == b || mode < 0 || mode > 15) return ZRX_EINVAL;
  // the link orders two streams of one device (events without a system fence, the low-
  // priority head stream beside the engine's own): both engines must be on it
  if (a->device != b->device) return ZRX_EINVAL;
  zrx_shard::DeviceGuard dg(a->device);
  for (zrx_ctx* c : {a, b}) {
    if (c->peer && c->peer != a && c->peer != b) { c->peer->peer = nullptr; c->peer->link_mode = 0; }
    // stream-to-stream on one device: no system-scope fence (which writes back the L2s)
    if (!c->ev_vit_done)
      ZRX_CHECK(hipEventCreateWithFlags(&c->ev_vit_done, hipEventDisableTiming | hipEventDisableSystemFence));
    if (!c->ev_chain_done)
      ZRX_CHECK(hipEventCreateWithFlags(&c->ev_chain_done, hipEventDisableTiming | hipEventDisableSystemFence));
    if ((mode & 4) && !c->lo) {
      int least = 0, greatest = 0;
      ZRX_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
      ZRX_CHECK(hipStreamCreateWithPriority(&c->lo, hipStreamNonBlocking, least));
      ZRX_CHECK(hipEventCreateWithFlags(&c->ev_lo_fork, hipEventDisableTiming | hipEventDisableSystemFence));
      ZRX_CHECK(hipEventCreateWithFlags(&c->ev_lo_join, hipEventDisableTiming | hipEventDisableSystemFence));
    }
  }
  a->peer = mode ? b : nullptr;
  b->peer = mode ? a : nullptr;
  a->link_mode = b->link_mode = mode;
  return ZRX_OK;
}

int zrx_enable_timing(zrx_ctx* c, int on) {
  if (!c) return ZRX_EINVAL;
  c->timing = on != 0;
  c->nrec = 0;
  // event sets for the first 64 timed launches are created here, not inside the timed region
  while (c->timing && c->evsets.size() < 64) {
    std::array<hipEvent_t, 6> set;
    for (auto& e : set) ZRX_CHECK(hipEventCreate(&e));
    c->evsets.push_back(set);
  }
  return ZRX_OK;
}

int zrx_get_timing(zrx_ctx* c, float* ms5) {
  if (!c || !ms5) return ZRX_EINVAL;
  for (int i = 0; i < 5; i++) ms5[i] = 0.f;
  if (c->nrec == 0) return ZRX_OK;
  ZRX_CHECK(hipEventSynchronize(c->evsets[c->nrec - 1][5]));
  for (size_t k = 0; k < c->nrec; k++)
    for (int i = 0; i < 5; i++) {
      float ms = 0.f;
      ZRX_CHECK(hipEventElapsedTime(&ms, c->evsets[k][i], c->evsets[k][i + 1]));
      ms5[i] += ms / (float)c->nrec;
    }
  c->nrec = 0;
  return ZRX_OK;
}

int zrx_reserve(zrx_ctx* c, int npkts, int max_nsym) {
  if (!c || npkts < 0 || max_nsym < 1) return ZRX_EINVAL;
  if (npkts <= c->cap_pkts && max_nsym <= c->cap_nsym) return ZRX_OK;
  zrx_shard::DeviceGuard dg(c->device);   // (the caller's device is restored on return)
  const int np = std::max(npkts, c->cap_pkts), ns = std::max(max_nsym, c->cap_nsym);
  free_ws(c);
  const int64_t stride = ((int64_t)std::max(ns - 1, 1) * 288 + 255) / 256 * 256;
  ZRX_CHECK(hipMalloc(&c->sig_soft, (size_t)np * 48 + 16));
  ZRX_CHECK(hipMalloc(&c->vparams, (size_t)np * 16 + 16));
  ZRX_CHECK(hipMalloc(&c->soft, (size_t)np * stride + 256));
  ZRX_CHECK(hipMalloc(&c->soft_off, (size_t)np * 8 + 8));
  ZRX_CHECK(hipMalloc(&c->dsym, (size_t)np * 4 + 8));
  ZRX_CHECK(hipMalloc(&c->wave_p0, ((size_t)np * std::max(ns - 1, 1) / 64 + 2) * 4));
  ZRX_CHECK(hipMalloc(&c->dec, (size_t)np * kDecStride + 256));
  ZRX_CHECK(hipMalloc(&c->dec_off, (size_t)np * 8 + 8));
  ZRX_CHECK(hipMalloc(&c->dec_bits, (size_t)np * 4 + 4));
  c->rows_cap = plan_rows_max(c, np);
  ZRX_CHECK(hipMalloc(&c->rows, (size_t)c->rows_cap * 8 + 8));
  ZRX_CHECK(hipMalloc(&c->nrows, v3::kPlanWords * 4));
  ZRX_CHECK(hipMemsetAsync(c->nrows, 0, v3::kPlanWords * 4, c->stream));   // (no plan to reuse)
  ZRX_CHECK(hipMalloc(&c->segs, (size_t)np + 16));
  ZRX_CHECK(hipMalloc(&c->order, (size_t)np * 4 + 16));
  ZRX_CHECK(hipMalloc(&c->dumps, (size_t)np * (v3::kMaxSeg - 1) * 2 * v3::kSeamWords * 8 + 256));
  const size_t nrec = (size_t)np / kPsBlock + 2;
  ZRX_CHECK(hipMalloc(&c->scan_rec, nrec * sizeof(PlanScanRec)));
  ZRX_CHECK(hipMalloc(&c->scan_ctr, 64));
  ZRX_CHECK(hipMemsetAsync(c->scan_rec, 0, nrec * sizeof(PlanScanRec), c->stream));
  ZRX_CHECK(hipMemsetAsync(c->scan_ctr, 0, 64, c->stream));
  if (np > 0) {
    k_fill_offsets<<<blocks(np, 256), 256, 0, c->stream>>>(c->soft_off, np, stride);
    k_fill_offsets<<<blocks(np, 256), 256, 0, c->stream>>>(c->dec_off, np, kDecStride);
    ZRX_CHECK(hipGetLastError());
  }
  ZRX_CHECK(hipStreamSynchronize(c->stream));
  c->cap_pkts = np; c->cap_nsym = ns; c->soft_stride = stride;
  return ZRX_OK;
}

int zrx_plan_stats(zrx_ctx* c, int32_t* stats2) {
  if (!c || !stats2) return ZRX_EINVAL;
  stats2[0] = stats2[1] = 0;
  if (!c->nrows) return ZRX_OK;
  ZRX_CHECK(hipMemcpyAsync(stats2, c->nrows, 8, hipMemcpyDeviceToHost, c->stream));
  ZRX_CHECK(hipStreamSynchronize(c->stream));
  return ZRX_OK;
}

#ifdef ZRX_VTRACE
int zrx_vtrace_set(void* p, int rows) {   // (timeline probe builds only) per-row trace buffer, 32 B per row slot
  const uint32_t n = p ? (uint32_t)std::max(rows, 0) : 0u;
  ZRX_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_vtrace_rows), &n, sizeof(n)));
  ZRX_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_vtrace), &p, sizeof(p)));
  return ZRX_OK;
}
#endif

int zrx_plan_check(zrx_ctx* c) {
  if (!c) return ZRX_EINVAL;
  if (!c->nrows) return ZRX_OK;
  int32_t h[8];
  ZRX_CHECK(hipMemcpyAsync(h, c->nrows, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  ZRX_CHECK(hipStreamSynchronize(c->stream));
  if (h[v3::kPlanDropped] != 0) {
    std::fprintf(stderr, "ziria_rx: the Viterbi plan dropped %d rows past its bound\n", h[v3::kPlanDropped]);
    return ZRX_EPLAN;
  }
  return ZRX_OK;
}

int zrx_fft64_dev(zrx_ctx* c, const struct complex16* d_in, struct complex16* d_out, int64_t nsym) {
  if (!c || nsym < 0 || (nsym > 0 && (!d_in || !d_out))) return ZRX_EINVAL;
  if (nsym == 0) return ZRX_OK;
  k_fft64<<<blocks(nsym, 256), 256, 0, c->stream>>>((const uint4*)d_in, (uint4*)d_out, nsym);
  ZRX_CHECK(hipGetLastError());
  return ZRX_OK;
}

int zrx_fft_dev(zrx_ctx* c, int nfft, const struct complex16* d_in, struct complex16* d_out, int64_t count) {
  if (!c || count < 0 || fftn_index(nfft) < 0 || (count > 0 && (!d_in || !d_out))) return ZRX_EINVAL;
  if (count == 0) return ZRX_OK;
  const int rc = fftn_plans(c);
  if (rc) return rc;
  launch_fft(c, nfft, d_in, d_out, count);
  ZRX_CHECK(hipGetLastError());
  return ZRX_OK;
}

int zrx_viterbi_dev(zrx_ctx* c, const int8_t* d_soft, const int64_t* d_soft_off, const int32_t* d_params,
                    int npkts, uint8_t* d_out, const int64_t* d_out_off, int32_t* d_out_bits) {
  if (!c || npkts < 0) return ZRX_EINVAL;
  if (npkts == 0) return ZRX_OK;
#ifdef ZRX_GUARD
  {
    const char* ob = std::getenv("ZRX_GUARD_OUT");
    const uint64_t lo = (uint64_t)(uintptr_t)d_out, hi = lo + (ob ? std::strtoull(ob, nullptr, 10) : 0ull);
    const uint32_t np = (uint32_t)npkts;
    ZRX_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(v3::g_zg_out_lo), &lo, 8));
    ZRX_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(v3::g_zg_out_hi), &hi, 8));
    ZRX_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(v3::g_zg_np), &np, 4));
  }
#endif
  const int rc = ws_acquire(c);
  if (rc) return rc;
  launch_viterbi(c, (const uint8_t*)d_soft, d_soft_off, d_params, npkts, d_out, d_out_off, d_out_bits);
  ZRX_CHECK(hipGetLastError());
  return ws_release(c);
}

static void* pinned_mapped(size_t bytes, void** dev);
static int rx_chain(zrx_ctx* c, const struct complex16* d_sym, const int64_t* d_sym_off, const int32_t* d_nsym,
                    int npkts, int max_nsym, const struct complex16* d_chan, uint8_t* d_payload, int32_t* d_info) {
  if (!c || npkts < 0 || max_nsym < 1) return ZRX_EINVAL;
  if (npkts > c->cap_pkts || max_nsym > c->cap_nsym) {
    std::fprintf(stderr, "ziria_rx: workspace holds %d packets x %d symbols, call zrx_reserve(%d, %d)\n",
                 c->cap_pkts, c->cap_nsym, npkts, max_nsym);
    return ZRX_ENOMEM;
  }
  if (npkts == 0) return ZRX_OK;
  EqTabs T{nullptr, nullptr};
  if (d_chan) {
    const int rc = ensure_eq_tables(c);
    if (rc) return rc;
    T = EqTabs{c->eq_rot, c->eq_atan};
  }
  {
    const int rc = ws_acquire(c);
    if (rc) return rc;
  }
  const uint32_t* chan = (const uint32_t*)d_chan;
  hipStream_t s = c->stream;
  // h: the stream of the chain's head (SIGNAL, plan, k_data_fft): the caller's, or with link
  // mode 4 a low-priority stream of the context, so that where two linked engines overlap the
  // other batch's Viterbi blocks are dispatched before this batch's head blocks.
  const bool lo = c->peer && (c->link_mode & 4) && c->lo;
  hipStream_t h = s;
  if (lo) {
    ZRX_CHECK(hipEventRecord(c->ev_lo_fork, s));
    ZRX_CHECK(hipStreamWaitEvent(c->lo, c->ev_lo_fork, 0));
    h = c->lo;
  }
  hipEvent_t* ev = nullptr;
  if (c->timing) {
    if (c->nrec == c->evsets.size()) {
      std::array<hipEvent_t, 6> set;
      for (auto& e : set) ZRX_CHECK(hipEventCreate(&e));
      c->evsets.push_back(set);
    }
    ev = c->evsets[c->nrec++].data();
  }
  if (ev) ZRX_CHECK(hipEventRecord(ev[0], h));
  // one lane per packet, kSigFftLanes packets per one-wave block.  (16 measured worse: 9.4 ->
  // 14.3 us at config 3, and with two engines in flight its 1024 single-wave blocks took CU
  // slots the other batch's Viterbi blocks were placed by: config 5 101 -> 76 Gbit/s.)
  if (chan)
    k_signal_fft<true><<<blocks(npkts, kSigFftLanes), kSigFftLanes, 0, h>>>((const uint4*)d_sym, d_sym_off, d_nsym,
                                                                            npkts, (uint4*)c->sig_soft, chan, T);
  else
    k_signal_fft<false><<<blocks(npkts, kSigFftLanes), kSigFftLanes, 0, h>>>((const uint4*)d_sym, d_sym_off, d_nsym,
                                                                             npkts, (uint4*)c->sig_soft, chan, T);
  if (ev) ZRX_CHECK(hipEventRecord(ev[1], h));
  const bool ordered = order_fits(c, npkts);
  k_signal_vit<<<blocks(npkts, v3::kRows), 256, 0, h>>>(c->sig_soft, d_nsym, npkts, c->cap_nsym, c->vparams, d_info,
                                                 ordered ? c->nrows : nullptr);
  // A mixed batch's sort and row expansion (k_pkt_rows) only feed the Viterbi, so they can run
  // on a side stream while k_data_fft runs (config 5: -27 us a batch).  The fork and join cost
  // ~19 us of queue latency (config 3: +19 us) and a uniform batch has nothing to sort, so the
  // plan is split only when the previous batch was mixed (k_pkt_plan writes that to a mapped
  // host word; a stale read only picks the slower path: either way the rows are exact).
  if (!c->mixed_hint) {
    void* dp = nullptr;
    c->mixed_hint = (int32_t*)pinned_mapped(64, &dp);
    if (!c->mixed_hint) return ZRX_ENOMEM;
    c->mixed_hint_dev = (int32_t*)dp;
    *(volatile int32_t*)c->mixed_hint = 0;
  }
  const bool split = ordered && *(volatile int32_t*)c->mixed_hint != 0;
  if (split) {                                         // forked before the plan: see k_pkt_rows
    if (!c->side) {
      ZRX_CHECK(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
      // (stream-to-stream on one device: no system-scope fence, which writes back the L2s)
      ZRX_CHECK(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming | hipEventDisableSystemFence));
      ZRX_CHECK(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming | hipEventDisableSystemFence));
    }
    ZRX_CHECK(hipEventRecord(c->ev_fork, h));
    ZRX_CHECK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
    k_pkt_rows<<<1, 1024, 0, c->side>>>(c->vparams, npkts, c->rows, c->nrows, c->segs, c->order, c->dec_bits, c->ncu,
                                        (int)plan_rows_max(c, npkts));
    ZRX_CHECK(hipEventRecord(c->ev_join, c->side));
  }
  // the plan: offsets, the batch verdict and (unless split) a mixed batch's rows, over many blocks
  if (++c->scan_epoch == 0) c->scan_epoch = 1;
  k_pkt_scan<<<blocks(npkts, kPsBlock), kPsThreads, 0, h>>>(
      c->vparams, npkts, c->soft_off, c->dsym, c->wave_p0, ordered ? c->rows : nullptr, ordered ? c->nrows : nullptr,
      c->segs, c->order, c->dec_bits, c->ncu, (int)plan_rows_max(c, npkts), split ? 1 : 0,
      ordered ? c->mixed_hint_dev : nullptr, c->scan_rec, c->scan_ctr, c->scan_epoch);
  if (ev) ZRX_CHECK(hipEventRecord(ev[2], h));
  // k_data_fft: waves over the batch's data symbols, at most npkts x (max_nsym - 1) of them
  const int fft_blocks = (int)std::min<int64_t>(((int64_t)npkts * (max_nsym - 1) + kDfThreads - 1) / kDfThreads,
                                                (int64_t)(chan ? c->df_blocks_eq : c->df_blocks));
  zrx_ctx* const peer = c->peer;
  // (a never-recorded peer event is complete: the first batch waits for nothing)
  if (peer && (c->link_mode & 2)) ZRX_CHECK(hipStreamWaitEvent(h, peer->ev_vit_done, 0));
  if (fft_blocks > 0) {
    if (chan)
      k_data_fft<true><<<fft_blocks, kDfThreads, 0, h>>>((const uint4*)d_sym, d_sym_off, c->vparams, npkts, (uint4*)c->soft,
                                                   c->soft_off, c->dsym, c->wave_p0, chan, T);
    else
      k_data_fft<false><<<fft_blocks, kDfThreads, 0, h>>>((const uint4*)d_sym, d_sym_off, c->vparams, npkts, (uint4*)c->soft,
                                                    c->soft_off, c->dsym, c->wave_p0, chan, T);
  }
  if (ev) ZRX_CHECK(hipEventRecord(ev[3], h));
  if (split) ZRX_CHECK(hipStreamWaitEvent(s, c->ev_join, 0));
  if (lo) {
    ZRX_CHECK(hipEventRecord(c->ev_lo_join, h));
    ZRX_CHECK(hipStreamWaitEvent(s, c->ev_lo_join, 0));
  }
  // (mode bit 3: only for the peer's Viterbi and seam pass, so its descramble/CRC overlaps the
  // start of this Viterbi)
  if (peer && (c->link_mode & 1))
    ZRX_CHECK(hipStreamWaitEvent(s, (c->link_mode & 8) ? peer->ev_vit_done : peer->ev_chain_done, 0));
  launch_viterbi(c, c->soft, c->soft_off, c->vparams, npkts, c->dec, c->dec_off, c->dec_bits, ordered);
  if (peer) ZRX_CHECK(hipEventRecord(c->ev_vit_done, s));
  if (ev) ZRX_CHECK(hipEventRecord(ev[4], s));
  k_descramble_crc<<<c->crc_blocks > 0 ? std::min(blocks(npkts, kCrcWaves), c->crc_blocks) : blocks(npkts, kCrcWaves),
                     64 * kCrcWaves, 0, s>>>(c->dec, c->dec_bits, d_info, d_payload, npkts);
  if (ev) ZRX_CHECK(hipEventRecord(ev[5], s));
  if (peer) ZRX_CHECK(hipEventRecord(c->ev_chain_done, s));
  ZRX_CHECK(hipGetLastError());
  return ws_release(c);
}

int zrx_rx_dev(zrx_ctx* c, const struct complex16* d_sym, const int64_t* d_sym_off, const int32_t* d_nsym,
               int npkts, int max_nsym, uint8_t* d_payload, int32_t* d_info) {
  return rx_chain(c, d_sym, d_sym_off, d_nsym, npkts, max_nsym, nullptr, d_payload, d_info);
}

int zrx_rx_eq_dev(zrx_ctx* c, const struct complex16* d_sym, const int64_t* d_sym_off, const int32_t* d_nsym,
                  int npkts, int max_nsym, const struct complex16* d_chan, uint8_t* d_payload, int32_t* d_info) {
  if (!d_chan && npkts > 0) return ZRX_EINVAL;
  return rx_chain(c, d_sym, d_sym_off, d_nsym, npkts, max_nsym, d_chan, d_payload, d_info);
}

int zrx_ofdm_eq_dev(zrx_ctx* c, const struct complex16* d_sym, const int64_t* d_sym_off, const int32_t* d_nsym,
                    int npkts, const struct complex16* d_chan, struct complex16* d_out) {
  if (!c || npkts < 0 || (npkts > 0 && (!d_sym || !d_sym_off || !d_nsym || !d_chan || !d_out))) return ZRX_EINVAL;
  if (npkts == 0) return ZRX_OK;
  const int rc = ensure_eq_tables(c);
  if (rc) return rc;
  k_ofdm_eq<<<blocks(npkts, 4), 256, 0, c->stream>>>((const uint4*)d_sym, d_sym_off, d_nsym, npkts,
                                                     (const uint32_t*)d_chan, EqTabs{c->eq_rot, c->eq_atan},
                                                     (uint4*)d_out);
  ZRX_CHECK(hipGetLastError());
  return ZRX_OK;
}

int zrx_rx_stream_dev(zrx_ctx* c, const struct complex16* d_samples, const int64_t* d_cap_off,
                      const int32_t* d_cap_len, int ncap, int max_len, int downsample, uint8_t* d_payload,
                      int32_t* d_info, int32_t* d_det) {
  if (!c || ncap < 0 || max_len < 0 || (ncap > 0 && (!d_samples || !d_cap_off || !d_cap_len || !d_payload ||
                                                     !d_info || !d_det)))
    return ZRX_EINVAL;
  if (ncap == 0) return ZRX_OK;
  const int n_max = downsample ? max_len / 8 * 4 : max_len;
  const int max_sym = std::max(1, n_max / 80);       // symbols after the LTS fit in the capture
  int rc = zrx_reserve(c, ncap, max_sym);
  if (rc) return rc;
  rc = ensure_eq_tables(c);
  if (rc) return rc;
  zrx_shard::DeviceGuard dg(c->device);   // (the caller's device is restored on return)
  if (!c->fe_pattern) {
    uint32_t pat[256];
    make_cca_pattern(pat);
    ZRX_CHECK(hipMalloc(&c->fe_pattern, sizeof(pat)));
    ZRX_CHECK(hipMemcpy(c->fe_pattern, pat, sizeof(pat), hipMemcpyHostToDevice));
  }
  if (ncap > c->fe_cap || max_sym > c->fe_sym) {
    for (void* p : {(void*)c->fe_syms, (void*)c->fe_sym_off, (void*)c->fe_nsym, (void*)c->fe_chan}) (void)hipFree(p);
    const int nc = std::max(ncap, c->fe_cap), ns = std::max(max_sym, c->fe_sym);
    ZRX_CHECK(hipMalloc(&c->fe_syms, (size_t)nc * ns * 256 + 256));
    ZRX_CHECK(hipMalloc(&c->fe_sym_off, (size_t)nc * 8 + 8));
    ZRX_CHECK(hipMalloc(&c->fe_nsym, (size_t)nc * 4 + 4));
    ZRX_CHECK(hipMalloc(&c->fe_chan, (size_t)nc * 256 + 256));
    c->fe_cap = nc; c->fe_sym = ns;
  }
  rc = ws_acquire(c);                                // the front-end staging is workspace too
  if (rc) return rc;
  const uint32_t* smp = (const uint32_t*)d_samples;
  hipStream_t s = c->stream;
  fe::k_fe_detect<<<blocks(ncap, 4), 256, 0, s>>>(smp, d_cap_off, d_cap_len, ncap, downsample, 1000, c->fe_pattern, d_det);
  fe::k_fe_lts<<<blocks(ncap, 64), 64, 0, s>>>(smp, d_cap_off, d_cap_len, ncap, downsample, d_det, make_agc_ties(),
                                              c->fe_chan);
  fe::k_fe_gather<<<blocks(ncap, 4), 256, 0, s>>>(smp, d_cap_off, d_cap_len, ncap, downsample, d_det, max_sym,
                                                  c->fe_syms, c->fe_sym_off, c->fe_nsym);
  ZRX_CHECK(hipGetLastError());
  return rx_chain(c, (const complex16*)c->fe_syms, c->fe_sym_off, c->fe_nsym, ncap, max_sym,
                  (const complex16*)c->fe_chan, d_payload, d_info);
}

int zrx_tx_dev(zrx_ctx* c, const uint8_t* d_in, const int64_t* d_in_off, int npkts, struct complex16* d_out,
               const int64_t* d_out_off, int32_t* d_nsamp) {
  if (!c || npkts < 0 || (npkts > 0 && (!d_in || !d_in_off || !d_out || !d_out_off || !d_nsamp))) return ZRX_EINVAL;
  if (npkts == 0) return ZRX_OK;
  zrx_shard::DeviceGuard dg(c->device);   // (the caller's device is restored on return)
  if (!c->tx_preamble) {
    uint32_t pre[640];
    make_tx_preamble(pre);
    ZRX_CHECK(hipMalloc(&c->tx_preamble, sizeof(pre)));
    ZRX_CHECK(hipMemcpy(c->tx_preamble, pre, sizeof(pre), hipMemcpyHostToDevice));
  }
  tx::k_tx<<<npkts, 64, 0, c->stream>>>(d_in, d_in_off, npkts, c->tx_preamble, (uint32_t*)d_out, d_out_off, d_nsamp);
  ZRX_CHECK(hipGetLastError());
  return ZRX_OK;
}

int zrx_tx_preamble(int16_t* out1280) {
  if (!out1280) return ZRX_EINVAL;
  uint32_t p[640];
  make_tx_preamble(p);
  std::memcpy(out1280, p, sizeof(p));
  return ZRX_OK;
}

int zrx_tx_samples(const uint8_t* hdr3) {
  if (!hdr3) return ZRX_EINVAL;
  const uint32_t hb = (uint32_t)hdr3[0] | ((uint32_t)hdr3[1] << 8) | ((uint32_t)hdr3[2] << 16);
  static const int nc_of[16] = {0, 0, 0, 0, 0, 0, 0, 0, 288, 192, 96, 48, 288, 192, 96, 48};
  static const int cr_of[16] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 2, 2, 2, 2};
  int nc = nc_of[hb & 0xF], cr = cr_of[hb & 0xF];
  if (!nc) { nc = 48; cr = 0; }                       // parsePLCPHeader default: BPSK 1/2
  const int nd = cr == 0 ? nc / 2 : cr == 1 ? nc * 2 / 3 : nc * 3 / 4;
  const int len = std::min((int)((hb >> 5) & 0xFFF), 2048), plen = std::max(len - 4, 0);
  return 640 + 160 * (1 + (16 + 8 * plen + 32 + 6 + nd - 1) / nd);
}

int zrx_cca_pattern(int16_t* pattern512) {
  if (!pattern512) return ZRX_EINVAL;
  uint32_t p[256];
  make_cca_pattern(p);
  std::memcpy(pattern512, p, sizeof(p));
  return ZRX_OK;
}

int zrx_trig_tables(int16_t* sin65536, int16_t* cos65536, int16_t* atan65536) {
  if (!sin65536 || !cos65536 || !atan65536) return ZRX_EINVAL;
  make_trig_tables(sin65536, cos65536, atan65536);
  return ZRX_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ batched externals (host arrays)
// The per-call externals (Part 1 of ziria_rx.h) run on the host: zrx_host.cpp.  The batched
// ones below split every call over the node's logical shards (zrx_shard.hpp): contiguous
// packet ranges, one engine context per shard on its own device, stream, copy streams and
// host thread, each writing its packets' outputs straight into the caller's arrays.
static std::mutex g_mu;                  // one batched call at a time (the reference's decoder is global too)

namespace {
struct Node {
  std::vector<int> want;                 // zrx_set_devices (empty: ZRX_DEVICES, else every gfx950 device)
  int64_t min_shard_bytes = zrx_shard::kMinShardBytes;
  bool resolved = false;
  std::vector<int> dev;                  // device of each logical shard
  std::vector<zrx_ctx*> ctx;             // its engine context, created on first use
  zrx_io::Pool* pool = nullptr;          // the shards' host threads (shards - 1 workers + the caller)
  zrx_shard::HostRegistry reg;           // caller arrays the library page-locked
  int last_shards = 0;                   // shards the last call ran on
};
Node g_node;
}  // namespace

static bool is_gfx950(int device) {
  hipDeviceProp_t prop;
  return hipGetDeviceProperties(&prop, device) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

// Drops every shard context (the calls are synchronous: nothing of theirs is in flight).
static void node_reset() {
  for (size_t k = 0; k < g_node.ctx.size(); k++)
    if (g_node.ctx[k]) zrx_destroy(g_node.ctx[k]);
  g_node.ctx.clear();
  g_node.dev.clear();
  delete g_node.pool;
  g_node.pool = nullptr;
  g_node.resolved = false;
}

// The logical shards: zrx_set_devices' list, else ZRX_DEVICES, else every visible gfx950
// device.  ZRX_ENODEV without one (the batched externals have no CPU path).
static int node_resolve() {
  if (g_node.resolved) return ZRX_OK;
  std::vector<int> d = g_node.want;
  if (d.empty()) d = zrx_shard::parse_devices(std::getenv("ZRX_DEVICES"));
  if (d.empty()) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
      (void)hipGetLastError();
      n = 0;
    }
    for (int i = 0; i < n; i++)
      if (is_gfx950(i)) d.push_back(i);
  }
  if (d.empty()) {
    std::fprintf(stderr, "ziria_rx: no gfx950 device: the batched externals run on the GPU (no CPU path)\n");
    return ZRX_ENODEV;
  }
  for (int x : d)
    if (check_device(x) != ZRX_OK) return ZRX_ENODEV;
  g_node.dev = d;
  g_node.ctx.assign(d.size(), nullptr);
  g_node.pool = new zrx_io::Pool((int)d.size());
  g_node.resolved = true;
  return ZRX_OK;
}

// Shard k's context (own non-blocking stream on its device), created on first use.  Distinct
// shards are created from distinct threads: each touches only its own slot.
static zrx_ctx* node_ctx(int k) {
  if (g_node.ctx[(size_t)k]) return g_node.ctx[(size_t)k];
  const int dev = g_node.dev[(size_t)k];
  zrx_shard::DeviceGuard dg(dev);
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  zrx_ctx* c = nullptr;
  if (zrx_create(&c, dev, s) != ZRX_OK) {
    (void)hipStreamDestroy(s);
    return nullptr;
  }
  c->owns_stream = true;
  return g_node.ctx[(size_t)k] = c;
}

// Splits a call of np packets (weight prefix: the input bytes before packet i) over the
// shards and runs body(ctx, p0, p1) for each range on its shard's device; merged as
// zrx_shard::run: the first error, else the sum of the bodies' counts.
template <class Prefix, class Body>
static int node_run(int np, Prefix prefix, Body&& body) {
  int rc = node_resolve();
  if (rc) return rc;
  const std::vector<int> cut = zrx_shard::split(np, prefix, (int)g_node.dev.size(), g_node.min_shard_bytes);
  g_node.last_shards = (int)cut.size() - 1;
  return zrx_shard::run(g_node.pool, cut, [&](int k, int p0, int p1) -> int {
    zrx_ctx* c = node_ctx(k);
    if (!c) return ZRX_ENODEV;
    zrx_shard::DeviceGuard dg(c->device);
    return body(c, p0, p1);
  });
}

static bool registered(const void* p, size_t n) { return g_node.reg.ensure(p, n, zrx_io::is_pinned); }

static void* staging(zrx_ctx* c, size_t bytes) {
  if (bytes > c->small_cap) {
    (void)hipFree(c->small);
    c->small = nullptr;
    size_t cap = std::max<size_t>(bytes, 1 << 20);
    if (hipMalloc(&c->small, cap) != hipSuccess) { c->small_cap = 0; return nullptr; }
    c->small_cap = cap;
  }
  return c->small;
}

// Pinned host memory mapped into the device's address space (coherent: the GPU does not
// cache it); the rx chain's mixed-batch hint word lives there.
static void* pinned_mapped(size_t bytes, void** dev) {
  void* h = nullptr;
  if (hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
  if (hipHostGetDevicePointer(dev, h, 0) != hipSuccess) { (void)hipHostFree(h); return nullptr; }
  return h;
}

#define ZRX_DIE(msg)                                                     \
  do {                                                                   \
    std::fprintf(stderr, "ziria_rx: %s (%s:%d)\n", msg, __FILE__, __LINE__); \
    std::abort();                                                        \
  } while (0)

namespace zrx_batch {

// The host pipelines' per-context state (zrx_hostio.hpp), created on first use; its copy pool
// gets this shard's share of the host threads.
static zrx_io::HostIO* host_io(zrx_ctx* c) {
  if (c->hio) return c->hio;
  auto* io = new zrx_io::HostIO();
  const unsigned hc = std::max(1u, std::thread::hardware_concurrency());
  const int share = (int)std::min<unsigned>(8u, std::max(1u, hc / 2 / (unsigned)std::max<size_t>(1, g_node.dev.size())));
  if (io->init(c->device, share) != hipSuccess) {
    std::fprintf(stderr, "ziria_rx: copy streams / events for the host pipeline could not be created\n");
    delete io;
    return nullptr;
  }
  return c->hio = io;
}

// Waits for everything a host pipeline issued, on its error paths too: no copy into or out
// of the caller's arrays may still be in flight when the call returns.
static void host_io_quiesce(zrx_ctx* c) {
  if (c->hio) {
    (void)hipStreamSynchronize(c->hio->up);
    (void)hipStreamSynchronize(c->hio->down);
  }
  (void)hipStreamSynchronize(c->stream);
}

// Plan words of the chunks (pinned: read back without a sync per chunk): any dropped row is
// ZRX_EPLAN, never silent.
static int plan_flags_ok(const zrx_io::HostIO* io, int nch) {
  for (int j = 0; j < nch; j++)
    if (io->flags[j] != 0) {
      std::fprintf(stderr, "ziria_rx: the Viterbi plan dropped %d rows past its bound\n", io->flags[j]);
      return ZRX_EPLAN;
    }
  return ZRX_OK;
}

// ---- FFT64 batch: symbols [q0, q1) of one shard
static int fft64_range(zrx_ctx* c, struct complex16* out, const struct complex16* in, int q0, int q1) {
  const size_t bytes = (size_t)(q1 - q0) * 256;
  uint8_t* d = (uint8_t*)staging(c, 2 * bytes);
  if (!d) return ZRX_ENOMEM;
  ZRX_CHECK(hipMemcpyAsync(d, (const uint8_t*)in + (size_t)q0 * 256, bytes, hipMemcpyHostToDevice, c->stream));
  const int rc = zrx_fft64_dev(c, (const complex16*)d, (complex16*)(d + bytes), q1 - q0);
  if (rc) return rc;
  ZRX_CHECK(hipMemcpyAsync((uint8_t*)out + (size_t)q0 * 256, d + bytes, bytes, hipMemcpyDeviceToHost, c->stream));
  ZRX_CHECK(hipStreamSynchronize(c->stream));
  return 0;
}

// nsym independent FFT64s (no return value to carry an error: fails loudly without a GPU)
void sora_fft64_batch(struct complex16* out, int outlen, struct complex16* in, int inlen) {
  if (inlen <= 0 || inlen % 64 || outlen < inlen) {
    std::fprintf(stderr, "ziria_rx: __ext_sora_fft64_batch needs inlen = 64*k and outlen >= inlen\n");
    return;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  const int rc = node_run(inlen / 64, [](int i) { return (int64_t)i * 256; },
                          [&](zrx_ctx* c, int q0, int q1) { return fft64_range(c, out, in, q0, q1); });
  if (rc == ZRX_ENODEV) ZRX_DIE("no gfx950 device: the batched externals run on the GPU");
  if (rc < 0) ZRX_DIE("__ext_sora_fft64_batch failed");
}

// ---- Viterbi batch
struct VitCall {
  const char* soft;
  const int32_t* soft_off;                 // n + 1 (validated: non-decreasing, within softlen)
  const int32_t* frame_len;
  const int16_t* code_rate;
  unsigned char* out;
  const int32_t* out_off;
  bool pin_in;
};

// Packets [q0, q1) of one shard: frame i decodes soft[soft_off[i] .. soft_off[i+1]) and its
// bytes land at out[out_off[i] ..].  The frames are decoded into a packed device buffer (frame
// i at the prefix of frame_len) and only the bytes each frame produced (out_bits_count / 8: the
// brick emits whole bytes, window by window) are scattered into the caller's array, whose other
// bytes stay as they were; so the caller's output array is never uploaded.  The shard's soft
// values go up in chunks (zrx_hostio.hpp) into a device copy of just its range.
static int vit_range(zrx_ctx* c, const VitCall& a, int q0, int q1) {
  const int np = q1 - q0;
  if (np <= 0) return 0;
  const int64_t base = a.soft_off[q0];
  std::vector<int32_t> params(4 * (size_t)np);
  std::vector<int64_t> soff(np), coff(np + 1);
  coff[0] = 0;
  for (int i = 0; i < np; i++) {
    const int g = q0 + i;
    params[4 * i] = a.frame_len[g];
    params[4 * i + 1] = a.code_rate[g];
    params[4 * i + 2] = a.soft_off[g + 1] - a.soft_off[g];
    params[4 * i + 3] = 0;
    soff[i] = a.soft_off[g] - base;
    coff[i + 1] = coff[i] + a.frame_len[g];
  }
  const auto sof = [&](int i) { return (size_t)(a.soft_off[q0 + i] - base); };   // local soft offset of packet i
  const std::vector<int> cut = zrx_io::chunk_cuts(np, [&](int i) { return sof(i + 1) - sof(i); }, sof(np));
  const int nch = (int)cut.size() - 1;
  int maxn = 0;
  size_t in_max = 0, out_max = 0;
  for (int j = 0; j < nch; j++) {
    const int n = cut[j + 1] - cut[j];
    maxn = std::max(maxn, n);
    in_max = std::max(in_max, sof(cut[j + 1]) - sof(cut[j]));
    out_max = std::max(out_max, (size_t)n * 4 + (size_t)(coff[cut[j + 1]] - coff[cut[j]]));
  }
  int rc = zrx_reserve(c, maxn, 1);                  // room for the row plan of k_pkt_plan
  if (rc) return rc;
  zrx_io::HostIO* io = host_io(c);
  if (!io) return ZRX_EHIP;
  const auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t s_soft = al(sof(np)), s_par = al((size_t)np * 16), s_off = al((size_t)np * 8);
  const size_t s_out = al((size_t)coff[np]);
  uint8_t* d = (uint8_t*)staging(c, s_soft + s_par + 2 * s_off + s_out + al((size_t)np * 4));
  if (!d) return ZRX_ENOMEM;
  uint8_t* d_soft = d;
  int32_t* d_par = (int32_t*)(d_soft + s_soft);
  int64_t* d_soff = (int64_t*)((uint8_t*)d_par + s_par);
  int64_t* d_coff = (int64_t*)((uint8_t*)d_soff + s_off);
  uint8_t* d_out = (uint8_t*)d_coff + s_off;
  int32_t* d_bits = (int32_t*)(d_out + s_out);
  const char* hsoft = a.soft + base;
  if ((!a.pin_in && io->reserve_in(in_max) != hipSuccess) || io->reserve_out(out_max) != hipSuccess ||
      io->reserve_flags(nch) != hipSuccess)
    return ZRX_ENOMEM;
  auto run = [&]() -> int {
    ZRX_CHECK(hipMemcpyAsync(d_par, params.data(), (size_t)np * 16, hipMemcpyHostToDevice, io->up));
    ZRX_CHECK(hipMemcpyAsync(d_soff, soff.data(), (size_t)np * 8, hipMemcpyHostToDevice, io->up));
    ZRX_CHECK(hipMemcpyAsync(d_coff, coff.data(), (size_t)np * 8, hipMemcpyHostToDevice, io->up));
    // chunk j's outputs, staged in out slot j & 1: packed bytes, then the bit counts
    auto drain = [&](int j) -> int {
      const int slot = j & 1, p0 = cut[j], p1 = cut[j + 1];
      ZRX_CHECK(hipEventSynchronize(io->down_done[slot]));
      const uint8_t* bytes = io->out[slot];
      const int32_t* bits = (const int32_t*)(bytes + (size_t)(coff[p1] - coff[p0]));
      io->pool->run((p1 - p0 + 255) / 256, [&](int t) {
        for (int i = p0 + 256 * t; i < std::min(p1, p0 + 256 * (t + 1)); i++) {
          const int nb = std::min<int>(a.frame_len[q0 + i], (std::max(bits[i - p0], 0) + 7) / 8);
          std::memcpy(a.out + a.out_off[q0 + i], bytes + (coff[i] - coff[p0]), (size_t)nb);
        }
      });
      return ZRX_OK;
    };
    for (int j = 0; j < nch; j++) {
      const int slot = j & 1, p0 = cut[j], p1 = cut[j + 1], n = p1 - p0;
      const size_t s0 = sof(p0), sb = sof(p1) - sof(p0);
      const char* src = hsoft + s0;
      if (!a.pin_in) {
        ZRX_CHECK(hipEventSynchronize(io->up_done[slot]));   // the slot's last upload is done
        zrx_io::par_copy(*io->pool, io->in[slot], src, sb);
        src = (const char*)io->in[slot];
      }
      if (sb) ZRX_CHECK(hipMemcpyAsync(d_soft + s0, src, sb, hipMemcpyHostToDevice, io->up));
      ZRX_CHECK(hipEventRecord(io->up_done[slot], io->up));
      ZRX_CHECK(hipStreamWaitEvent(c->stream, io->up_done[slot], 0));
      const int r = zrx_viterbi_dev(c, (const int8_t*)d_soft, d_soff + p0, d_par + 4 * (size_t)p0, n, d_out,
                                    d_coff + p0, d_bits + p0);
      if (r) return r;
      ZRX_CHECK(hipMemcpyAsync(io->flags + j, c->nrows + v3::kPlanDropped, 4, hipMemcpyDeviceToHost, c->stream));
      ZRX_CHECK(hipEventRecord(io->decoded, c->stream));
      ZRX_CHECK(hipStreamWaitEvent(io->down, io->decoded, 0));
      const size_t ob = (size_t)(coff[p1] - coff[p0]);
      if (ob) ZRX_CHECK(hipMemcpyAsync(io->out[slot], d_out + coff[p0], ob, hipMemcpyDeviceToHost, io->down));
      ZRX_CHECK(hipMemcpyAsync(io->out[slot] + ob, d_bits + p0, (size_t)n * 4, hipMemcpyDeviceToHost, io->down));
      ZRX_CHECK(hipEventRecord(io->down_done[slot], io->down));
      if (j >= 1) {
        const int r2 = drain(j - 1);                   // (overlaps chunk j's transfers and decode)
        if (r2) return r2;
      }
    }
    return drain(nch - 1);
  };
  rc = run();
  host_io_quiesce(c);
  if (rc) return rc;
  rc = plan_flags_ok(io, nch);
  return rc ? rc : np;
}

int32_t viterbi_batch_decode(const char* soft, int softlen, const int32_t* pkt_soft_off, int n_off,
                             const int32_t* frame_len, int n_fl, const int16_t* code_rate, int n_cr,
                             unsigned char* out_bits, int out_len_bits, const int32_t* pkt_out_off, int n_oo) {
  const int np = n_off - 1;
  if (np < 0 || n_fl < np || n_cr < np || n_oo < np || softlen < 0 || out_len_bits < 0) return ZRX_EINVAL;
  if (np == 0) return 0;
  const int64_t out_bytes = out_len_bits / 8;
  for (int i = 0; i < np; i++) {
    const int32_t n = pkt_soft_off[i + 1] - pkt_soft_off[i];
    const int cr = code_rate[i];
    if (cr < 0 || cr > 2 || n < 0 || n % 48 || pkt_soft_off[i] < 0 || pkt_soft_off[i + 1] > softlen ||
        frame_len[i] < 0 || frame_len[i] > 4990 || pkt_out_off[i] < 0 || pkt_out_off[i] + (int64_t)frame_len[i] > out_bytes)
      return ZRX_EINVAL;
  }
  // the frames' output ranges must not overlap: the shards (and each shard's copy threads)
  // write them concurrently
  {
    std::vector<int> ord;
    ord.reserve(np);
    for (int i = 0; i < np; i++)
      if (frame_len[i] > 0) ord.push_back(i);
    std::sort(ord.begin(), ord.end(), [&](int x, int y) { return pkt_out_off[x] < pkt_out_off[y]; });
    for (size_t k = 1; k < ord.size(); k++)
      if ((int64_t)pkt_out_off[ord[k - 1]] + frame_len[ord[k - 1]] > pkt_out_off[ord[k]]) {
        std::fprintf(stderr, "ziria_rx: __ext_viterbi_batch_decode: output ranges of frames %d and %d overlap\n",
                     ord[k - 1], ord[k]);
        return ZRX_EINVAL;
      }
  }
  std::lock_guard<std::mutex> lk(g_mu);
  const int rc0 = node_resolve();
  if (rc0) return rc0;
  VitCall a{soft, pkt_soft_off, frame_len, code_rate, out_bits, pkt_out_off, false};
  a.pin_in = registered(soft + pkt_soft_off[0], (size_t)(pkt_soft_off[np] - pkt_soft_off[0]));
  return node_run(np, [&](int i) { return (int64_t)pkt_soft_off[i]; },
                  [&](zrx_ctx* c, int q0, int q1) { return vit_range(c, a, q0, q1); });
}

// ---- receiveBits batch
struct RxCall {
  const uint8_t* sym;                      // 256 B per symbol
  const int32_t* sym_off;                  // n + 1 (validated)
  const uint8_t* chan;                     // 256 B per packet, or nullptr
  unsigned char* payload;                  // kPayloadStride B per packet
  int32_t* info;                           // 8 per packet
  bool pin_in, pin_out;
};

// Packets [q0, q1) of one shard: chunks of whole packets are uploaded, decoded and downloaded
// in a pipeline (zrx_hostio.hpp), the device holding only this shard's symbols.  A chunk's
// payload slots come back `cw` bytes wide: the most a packet of that chunk can carry (LENGTH -
// 4 <= 27 x data symbols - 6 at 54 Mbps, 216 bits a symbol for LENGTH + 2 decoded bytes;
// <= 2044 since LENGTH <= 2048), which k_descramble_crc writes in whole dwords after the
// chunk's memset zeroes them; a slot's bytes past cw keep the caller's contents.
static int rx_range(zrx_ctx* c, const RxCall& a, int q0, int q1) {
  const int np = q1 - q0;
  if (np <= 0) return 0;
  const int64_t base = a.sym_off[q0];
  std::vector<int64_t> off(np);
  std::vector<int32_t> ns(np);
  int max_ns = 1;
  for (int i = 0; i < np; i++) {
    off[i] = a.sym_off[q0 + i] - base;
    ns[i] = a.sym_off[q0 + i + 1] - a.sym_off[q0 + i];
    max_ns = std::max(max_ns, ns[i]);
  }
  const size_t cb = a.chan ? 256 : 0;                // channel bytes per packet
  const int64_t nsym = a.sym_off[q1] - base;
  const std::vector<int> cut = zrx_io::chunk_cuts(np, [&](int i) { return (size_t)ns[i] * 256 + cb; },
                                                   (size_t)nsym * 256 + cb * np);
  const int nch = (int)cut.size() - 1;
  std::vector<int> cmax(nch, 1), cw(nch, 0);
  int maxn = 0;
  size_t in_max = 0, out_max = 0;
  for (int j = 0; j < nch; j++) {
    const int n = cut[j + 1] - cut[j];
    for (int i = cut[j]; i < cut[j + 1]; i++) cmax[j] = std::max(cmax[j], ns[i]);
    cw[j] = (std::min(2044, std::max(27 * (cmax[j] - 1) - 6, 0)) + 3) & ~3;
    maxn = std::max(maxn, n);
    const int64_t s0 = j + 1 < nch ? off[cut[j + 1]] : nsym;
    in_max = std::max(in_max, (size_t)(s0 - off[cut[j]]) * 256 + cb * n);
    out_max = std::max(out_max, (size_t)n * 32 + (size_t)n * cw[j]);
  }
  int rc = zrx_reserve(c, maxn, max_ns);
  if (rc) return rc;
  zrx_io::HostIO* io = host_io(c);
  if (!io) return ZRX_EHIP;
  const auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t s_sym = al((size_t)nsym * 256) + 256;
  const size_t s_off = al((size_t)np * 8), s_ns = al((size_t)np * 4);
  const size_t s_pay = (size_t)np * kPayloadStride, s_info = al((size_t)np * 32);
  const size_t s_chan = (size_t)np * cb;
  uint8_t* d = (uint8_t*)staging(c, s_sym + s_off + s_ns + s_pay + s_info + s_chan);
  if (!d) return ZRX_ENOMEM;
  uint8_t* d_sym = d;
  int64_t* d_off = (int64_t*)(d + s_sym);
  int32_t* d_ns = (int32_t*)((uint8_t*)d_off + s_off);
  uint8_t* d_pay = (uint8_t*)d_ns + s_ns;
  int32_t* d_info = (int32_t*)(d_pay + s_pay);
  uint8_t* d_chan = (uint8_t*)d_info + s_info;
  const uint8_t* hs = a.sym + (size_t)base * 256;
  const uint8_t* hchan = a.chan ? a.chan + (size_t)q0 * 256 : nullptr;
  unsigned char* payload = a.payload + (size_t)q0 * kPayloadStride;
  int32_t* pkt_info = a.info + 8 * (size_t)q0;
  if ((!a.pin_in && io->reserve_in(in_max) != hipSuccess) || (!a.pin_out && io->reserve_out(out_max) != hipSuccess) ||
      io->reserve_flags(nch) != hipSuccess)
    return ZRX_ENOMEM;
  auto run = [&]() -> int {
    ZRX_CHECK(hipMemcpyAsync(d_off, off.data(), (size_t)np * 8, hipMemcpyHostToDevice, io->up));
    ZRX_CHECK(hipMemcpyAsync(d_ns, ns.data(), (size_t)np * 4, hipMemcpyHostToDevice, io->up));
    // chunk j's outputs, staged in out slot j & 1 (pageable caller arrays): info, then the
    // payload slots packed cw[j] bytes apart
    auto drain = [&](int j) -> int {
      const int slot = j & 1, p0 = cut[j], n = cut[j + 1] - p0;
      ZRX_CHECK(hipEventSynchronize(io->down_done[slot]));
      std::memcpy(pkt_info + 8 * (size_t)p0, io->out[slot], (size_t)n * 32);
      zrx_io::par_copy_2d(*io->pool, payload + (size_t)p0 * kPayloadStride, kPayloadStride,
                          io->out[slot] + (size_t)n * 32, cw[j], cw[j], n);
      return ZRX_OK;
    };
    for (int j = 0; j < nch; j++) {
      const int slot = j & 1, p0 = cut[j], p1 = cut[j + 1], n = p1 - p0;
      const size_t s0 = (size_t)off[p0] * 256, sb = (size_t)((p1 < np ? off[p1] : nsym) - off[p0]) * 256;
      const uint8_t* src = hs + s0;
      const uint8_t* csrc = hchan ? hchan + (size_t)p0 * 256 : nullptr;
      if (!a.pin_in) {
        ZRX_CHECK(hipEventSynchronize(io->up_done[slot]));   // the slot's last upload is done
        zrx_io::par_copy(*io->pool, io->in[slot], src, sb);
        if (csrc) std::memcpy(io->in[slot] + sb, csrc, (size_t)n * 256);
        src = io->in[slot];
        csrc = csrc ? io->in[slot] + sb : nullptr;
      }
      if (sb) ZRX_CHECK(hipMemcpyAsync(d_sym + s0, src, sb, hipMemcpyHostToDevice, io->up));
      if (csrc) ZRX_CHECK(hipMemcpyAsync(d_chan + (size_t)p0 * 256, csrc, (size_t)n * 256, hipMemcpyHostToDevice, io->up));
      ZRX_CHECK(hipEventRecord(io->up_done[slot], io->up));
      ZRX_CHECK(hipStreamWaitEvent(c->stream, io->up_done[slot], 0));
      uint8_t* dp = d_pay + (size_t)p0 * kPayloadStride;
      if (cw[j]) ZRX_CHECK(hipMemset2DAsync(dp, kPayloadStride, 0, cw[j], n, c->stream));
      const int r = rx_chain(c, (const complex16*)d_sym, d_off + p0, d_ns + p0, n, cmax[j],
                             hchan ? (const complex16*)(d_chan + (size_t)p0 * 256) : nullptr, dp,
                             d_info + 8 * (size_t)p0);
      if (r) return r;
      ZRX_CHECK(hipMemcpyAsync(io->flags + j, c->nrows + v3::kPlanDropped, 4, hipMemcpyDeviceToHost, c->stream));
      ZRX_CHECK(hipEventRecord(io->decoded, c->stream));
      ZRX_CHECK(hipStreamWaitEvent(io->down, io->decoded, 0));
      uint8_t* oi = a.pin_out ? (uint8_t*)(pkt_info + 8 * (size_t)p0) : io->out[slot];
      uint8_t* op = a.pin_out ? payload + (size_t)p0 * kPayloadStride : io->out[slot] + (size_t)n * 32;
      ZRX_CHECK(hipMemcpyAsync(oi, d_info + 8 * (size_t)p0, (size_t)n * 32, hipMemcpyDeviceToHost, io->down));
      if (cw[j])
        ZRX_CHECK(hipMemcpy2DAsync(op, a.pin_out ? (size_t)kPayloadStride : (size_t)cw[j], dp, kPayloadStride, cw[j],
                                   n, hipMemcpyDeviceToHost, io->down));
      ZRX_CHECK(hipEventRecord(io->down_done[slot], io->down));
      if (!a.pin_out && j >= 1) {
        const int r2 = drain(j - 1);                   // (overlaps chunk j's transfers and decode)
        if (r2) return r2;
      }
    }
    return a.pin_out ? ZRX_OK : drain(nch - 1);
  };
  rc = run();
  host_io_quiesce(c);
  if (rc) return rc;
  rc = plan_flags_ok(io, nch);
  if (rc) return rc;
  // every CRC-passing payload fits the bytes its chunk brought back (cw): a kernel writing
  // more than 216 bits a data symbol would otherwise hand back a cut payload marked good
  int ok = 0;
  for (int j = 0; j < nch; j++)
    for (int i = cut[j]; i < cut[j + 1]; i++) {
      const int32_t* inf = pkt_info + 8 * (size_t)i;
      if (inf[4] == 0) continue;
      if (inf[2] - 4 > cw[j]) {
        std::fprintf(stderr, "ziria_rx: packet %d carries %d payload bytes, past the %d its chunk returned\n", q0 + i,
                     inf[2] - 4, cw[j]);
        return ZRX_EINTERNAL;
      }
      ok++;
    }
  return ok;
}

int32_t wifi_rx_batch(struct complex16* sym, int nsym_total, const int32_t* pkt_sym_off, int n_off,
                      const struct complex16* chan, int chan_len, unsigned char* payload, int payload_len_bits,
                      int32_t* pkt_info, int n_info) {
  const int np = n_off - 1;
  if (np < 0 || nsym_total < 0 || n_info < 8 * np || (int64_t)payload_len_bits / 8 < (int64_t)np * kPayloadStride)
    return ZRX_EINVAL;
  if (chan && chan_len < 64 * (int64_t)np) return ZRX_EINVAL;
  if (np == 0) return 0;
  for (int i = 0; i < np; i++)
    if (pkt_sym_off[i] < 0 || pkt_sym_off[i + 1] < pkt_sym_off[i] || pkt_sym_off[i + 1] > nsym_total) return ZRX_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  const int rc0 = node_resolve();
  if (rc0) return rc0;
  const uint8_t* hs = (const uint8_t*)sym;
  RxCall a{hs, pkt_sym_off, (const uint8_t*)chan, payload, pkt_info, false, false};
  a.pin_in = registered(hs + (size_t)pkt_sym_off[0] * 256, (size_t)(pkt_sym_off[np] - pkt_sym_off[0]) * 256) &&
             (!chan || registered(chan, (size_t)np * 256));
  a.pin_out = registered(payload, (size_t)np * kPayloadStride) && registered(pkt_info, (size_t)np * 32);
  const size_t cb = chan ? 256 : 0;
  return node_run(np, [&](int i) { return (int64_t)pkt_sym_off[i] * 256 + (int64_t)cb * i; },
                  [&](zrx_ctx* c, int q0, int q1) { return rx_range(c, a, q0, q1); });
}

// ---- receiver() batch over captures [q0, q1) of one shard: the device holds only its samples
struct StreamCall {
  const uint8_t* samples;                  // 4 B per sample
  const int32_t* cap_off;                  // n + 1 (validated)
  int downsample;
  unsigned char* payload;
  int32_t* info;
  int32_t* det;
};

static int stream_range(zrx_ctx* c, const StreamCall& a, int q0, int q1) {
  const int nc = q1 - q0;
  if (nc <= 0) return 0;
  const int64_t base = a.cap_off[q0], nsamp = a.cap_off[q1] - base;
  std::vector<int64_t> off(nc);
  std::vector<int32_t> len(nc);
  int max_len = 0;
  for (int i = 0; i < nc; i++) {
    off[i] = a.cap_off[q0 + i] - base;
    len[i] = a.cap_off[q0 + i + 1] - a.cap_off[q0 + i];
    max_len = std::max(max_len, len[i]);
  }
  const auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t s_smp = al((size_t)nsamp * 4) + 256;
  const size_t s_off = al((size_t)nc * 8), s_len = al((size_t)nc * 4);
  const size_t s_pay = (size_t)nc * kPayloadStride, s_info = al((size_t)nc * 32);
  const size_t s_det = (size_t)nc * 4 * fe::kDetWords;
  uint8_t* d = (uint8_t*)staging(c, s_smp + s_off + s_len + s_pay + s_info + s_det + 1024);
  if (!d) return ZRX_ENOMEM;
  uint8_t* d_smp = d;
  int64_t* d_off = (int64_t*)(d + s_smp);
  int32_t* d_len = (int32_t*)((uint8_t*)d_off + s_off);
  uint8_t* d_pay = (uint8_t*)d_len + s_len;
  int32_t* d_info = (int32_t*)(d_pay + s_pay);
  int32_t* d_det = (int32_t*)((uint8_t*)d_info + s_info);
  unsigned char* payload = a.payload + (size_t)q0 * kPayloadStride;
  int32_t* info = a.info + 8 * (size_t)q0;
  int32_t* det = a.det + (size_t)fe::kDetWords * q0;
  auto run = [&]() -> int {
    ZRX_CHECK(hipMemcpyAsync(d_smp, a.samples + (size_t)base * 4, (size_t)nsamp * 4, hipMemcpyHostToDevice, c->stream));
    ZRX_CHECK(hipMemcpyAsync(d_off, off.data(), (size_t)nc * 8, hipMemcpyHostToDevice, c->stream));
    ZRX_CHECK(hipMemcpyAsync(d_len, len.data(), (size_t)nc * 4, hipMemcpyHostToDevice, c->stream));
    ZRX_CHECK(hipMemsetAsync(d_pay, 0, s_pay, c->stream));
    const int r = zrx_rx_stream_dev(c, (const complex16*)d_smp, d_off, d_len, nc, max_len, a.downsample, d_pay,
                                    d_info, d_det);
    if (r) return r;
    ZRX_CHECK(hipMemcpyAsync(payload, d_pay, s_pay, hipMemcpyDeviceToHost, c->stream));
    ZRX_CHECK(hipMemcpyAsync(info, d_info, (size_t)nc * 32, hipMemcpyDeviceToHost, c->stream));
    ZRX_CHECK(hipMemcpyAsync(det, d_det, s_det, hipMemcpyDeviceToHost, c->stream));
    return ZRX_OK;
  };
  int rc = run();
  (void)hipStreamSynchronize(c->stream);             // (nothing in flight on any return)
  if (rc) return rc;
  rc = zrx_plan_check(c);                            // rows dropped by the plan: ZRX_EPLAN, never silent
  if (rc) return rc;
  int ok = 0;
  for (int i = 0; i < nc; i++) ok += det[fe::kDetWords * i] && info[8 * i + 4] != 0;
  return ok;
}

int32_t wifi_rx_stream_batch(struct complex16* samples, int nsamples, const int32_t* cap_off, int n_off,
                             int downsample, unsigned char* payload, int payload_len_bits,
                             int32_t* pkt_info, int n_info, int32_t* det, int n_det) {
  const int nc = n_off - 1;
  if (nc < 0 || nsamples < 0 || n_info < 8 * nc || n_det < fe::kDetWords * nc ||
      (int64_t)payload_len_bits / 8 < (int64_t)nc * kPayloadStride)
    return ZRX_EINVAL;
  if (nc == 0) return 0;
  for (int i = 0; i < nc; i++)
    if (cap_off[i] < 0 || cap_off[i + 1] < cap_off[i] || cap_off[i + 1] > nsamples) return ZRX_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  const StreamCall a{(const uint8_t*)samples, cap_off, downsample, payload, pkt_info, det};
  return node_run(nc, [&](int i) { return (int64_t)cap_off[i] * 4; },
                  [&](zrx_ctx* c, int q0, int q1) { return stream_range(c, a, q0, q1); });
}

// ---- transmitter() batch over packets [q0, q1) of one shard
struct TxCall {
  const unsigned char* in;
  const int32_t* in_off;                   // n + 1 (validated)
  struct complex16* out;
  const int32_t* out_off;                  // n + 1 (filled by the call)
};

static int tx_range(zrx_ctx* c, const TxCall& a, int q0, int q1) {
  const int np = q1 - q0;
  if (np <= 0) return 0;
  const int64_t ib = a.in_off[q0], ob = a.out_off[q0];
  const int64_t in_bytes = a.in_off[q1] - ib, nsamp = a.out_off[q1] - ob;
  std::vector<int64_t> ioff(np), ooff(np);
  for (int i = 0; i < np; i++) {
    ioff[i] = a.in_off[q0 + i] - ib;
    ooff[i] = a.out_off[q0 + i] - ob;
  }
  const auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t s_in = al((size_t)in_bytes) + 256, s_off = al((size_t)np * 8);
  const size_t s_out = (size_t)nsamp * 4;
  uint8_t* d = (uint8_t*)staging(c, s_in + 2 * s_off + al((size_t)np * 4) + s_out + 1024);
  if (!d) return ZRX_ENOMEM;
  uint8_t* d_in = d;
  int64_t* d_ioff = (int64_t*)(d + s_in);
  int64_t* d_ooff = (int64_t*)((uint8_t*)d_ioff + s_off);
  int32_t* d_ns = (int32_t*)((uint8_t*)d_ooff + s_off);
  uint8_t* d_out = (uint8_t*)d_ns + al((size_t)np * 4);
  auto run = [&]() -> int {
    ZRX_CHECK(hipMemcpyAsync(d_in, a.in + ib, (size_t)in_bytes, hipMemcpyHostToDevice, c->stream));
    ZRX_CHECK(hipMemcpyAsync(d_ioff, ioff.data(), (size_t)np * 8, hipMemcpyHostToDevice, c->stream));
    ZRX_CHECK(hipMemcpyAsync(d_ooff, ooff.data(), (size_t)np * 8, hipMemcpyHostToDevice, c->stream));
    const int r = zrx_tx_dev(c, d_in, d_ioff, np, (complex16*)d_out, d_ooff, d_ns);
    if (r) return r;
    ZRX_CHECK(hipMemcpyAsync((uint8_t*)a.out + (size_t)ob * 4, d_out, s_out, hipMemcpyDeviceToHost, c->stream));
    return ZRX_OK;
  };
  const int rc = run();
  (void)hipStreamSynchronize(c->stream);             // (nothing in flight on any return)
  return rc ? rc : (int)nsamp;
}

int32_t wifi_tx_batch(const unsigned char* in, int inlen, const int32_t* pkt_in_off, int n_off,
                      struct complex16* out, int outlen, int32_t* pkt_out_off, int n_oo) {
  const int np = n_off - 1;
  if (np < 0 || inlen < 0 || n_oo < np + 1) return ZRX_EINVAL;
  if (np == 0) { pkt_out_off[0] = 0; return 0; }
  int64_t total = 0;
  for (int i = 0; i < np; i++) {
    if (pkt_in_off[i] < 0 || pkt_in_off[i + 1] - pkt_in_off[i] < 3 || pkt_in_off[i + 1] > inlen) return ZRX_EINVAL;
    const uint8_t* h = in + pkt_in_off[i];
    const int len = std::min((int)((((uint32_t)h[1] << 8 | h[0]) >> 5 | (uint32_t)h[2] << 11) & 0xFFF), 2048);
    if (pkt_in_off[i] + 3 + std::max(len - 4, 0) > pkt_in_off[i + 1]) return ZRX_EINVAL;   // payload bytes present
    pkt_out_off[i] = (int32_t)total;
    total += zrx_tx_samples(h);
    if (total > outlen) return ZRX_EINVAL;
  }
  pkt_out_off[np] = (int32_t)total;
  std::lock_guard<std::mutex> lk(g_mu);
  const TxCall a{in, pkt_in_off, out, pkt_out_off};
  return node_run(np, [&](int i) { return (int64_t)pkt_out_off[i] * 4; },
                  [&](zrx_ctx* c, int q0, int q1) { return tx_range(c, a, q0, q1); });
}

}  // namespace zrx_batch

// C linkage (ctypes, C callers); zrx_ext_cxx.cpp exports the same with C++ linkage
extern "C" {

void __ext_sora_fft64_batch(struct complex16* out, int outlen, struct complex16* in, int inlen) {
  zrx_batch::sora_fft64_batch(out, outlen, in, inlen);
}
int32_t __ext_viterbi_batch_decode(char* soft, int softlen, int32_t* pkt_soft_off, int n_off,
                                   int32_t* frame_len, int n_fl, int16_t* code_rate, int n_cr,
                                   unsigned char* out_bits, int out_len_bits, int32_t* pkt_out_off, int n_oo) {
  return zrx_batch::viterbi_batch_decode(soft, softlen, pkt_soft_off, n_off, frame_len, n_fl, code_rate, n_cr,
                                         out_bits, out_len_bits, pkt_out_off, n_oo);
}
int32_t __ext_wifi_rx_batch(struct complex16* sym, int nsym_total, int32_t* pkt_sym_off, int n_off,
                            unsigned char* payload, int payload_len_bits, int32_t* pkt_info, int n_info) {
  return zrx_batch::wifi_rx_batch(sym, nsym_total, pkt_sym_off, n_off, nullptr, 0, payload, payload_len_bits,
                                  pkt_info, n_info);
}
int32_t __ext_wifi_rx_eq_batch(struct complex16* sym, int nsym_total, int32_t* pkt_sym_off, int n_off,
                               struct complex16* chan, int chan_len, unsigned char* payload, int payload_len_bits,
                               int32_t* pkt_info, int n_info) {
  if (!chan) return ZRX_EINVAL;
  return zrx_batch::wifi_rx_batch(sym, nsym_total, pkt_sym_off, n_off, chan, chan_len, payload, payload_len_bits,
                                  pkt_info, n_info);
}
int32_t __ext_wifi_rx_stream_batch(struct complex16* samples, int nsamples, int32_t* cap_off, int n_off,
                                   int downsample, unsigned char* payload, int payload_len_bits,
                                   int32_t* pkt_info, int n_info, int32_t* det, int n_det) {
  return zrx_batch::wifi_rx_stream_batch(samples, nsamples, cap_off, n_off, downsample, payload, payload_len_bits,
                                         pkt_info, n_info, det, n_det);
}
int32_t __ext_wifi_tx_batch(unsigned char* in, int inlen, int32_t* pkt_in_off, int n_off,
                            struct complex16* out, int outlen, int32_t* pkt_out_off, int n_oo) {
  return zrx_batch::wifi_tx_batch(in, inlen, pkt_in_off, n_off, out, outlen, pkt_out_off, n_oo);
}

// ---- the node behind the batched externals
int zrx_set_devices(const int32_t* devices, int n, int64_t min_shard_bytes) {
  if (n < 0 || (n > 0 && !devices)) return ZRX_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  for (int i = 0; i < n; i++)
    if (check_device(devices[i]) != ZRX_OK) return ZRX_ENODEV;
  node_reset();
  g_node.want.assign(devices, devices + n);
  g_node.min_shard_bytes = min_shard_bytes < 0 ? zrx_shard::kMinShardBytes : min_shard_bytes;
  return ZRX_OK;
}

int zrx_get_devices(int32_t* devices, int cap) {
  if (cap < 0 || (cap > 0 && !devices)) return ZRX_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  const int rc = node_resolve();
  if (rc) return rc;
  for (int i = 0; i < std::min(cap, (int)g_node.dev.size()); i++) devices[i] = g_node.dev[(size_t)i];
  return (int)g_node.dev.size();
}

int zrx_node_stats(int64_t* stats8) {
  if (!stats8) return ZRX_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  stats8[0] = g_node.last_shards;
  g_node.reg.stats(stats8 + 1);
  stats8[7] = (int64_t)g_node.min_shard_bytes;
  return ZRX_OK;
}

int zrx_set_host_register(int mode) {
  if (mode < 0 || mode > 2) return ZRX_EINVAL;
  std::lock_guard<std::mutex> lk(g_mu);
  g_node.reg.set_mode(mode);
  return ZRX_OK;
}

int zrx_shard_split(const int64_t* prefix, int np, int nshards, int64_t min_bytes, int32_t* cut) {
  if (np < 0 || nshards < 1 || !cut || (np > 0 && !prefix)) return ZRX_EINVAL;
  for (int i = 0; i < np; i++)
    if (prefix[i + 1] < prefix[i]) return ZRX_EINVAL;
  const std::vector<int> c = zrx_shard::split(np, [&](int i) { return prefix[i]; }, nshards, min_bytes);
  for (size_t k = 0; k < c.size(); k++) cut[k] = c[k];
  return (int)c.size() - 1;
}

int zrx_shard_selftest(const int64_t* prefix, int np, int nshards, int64_t min_bytes, int32_t* owner,
                       int fail_shard) {
  if (np < 0 || nshards < 1 || !owner || (np > 0 && !prefix)) return ZRX_EINVAL;
  const std::vector<int> cut = zrx_shard::split(np, [&](int i) { return prefix[i]; }, nshards, min_bytes);
  zrx_io::Pool pool(nshards);
  return zrx_shard::run(&pool, cut, [&](int k, int p0, int p1) -> int {
    if (k == fail_shard) return ZRX_EINTERNAL;
    for (int i = p0; i < p1; i++) owner[i] = k;
    return p1 - p0;
  });
}

}  // extern "C"
