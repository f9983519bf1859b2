/*
 * ORACLE — test infrastructure only.
 *
 * Sanitizer self-test of the C restatement (SURVEY.md §5 "Race detection / sanitizers"):
 * built with -fsanitize=address,undefined by `make -C oracle asan` and run on the CPU.  It
 * drives every oracle entry point the parity tests use, on round trips whose answers are
 * known without a GPU (transmit -> receive of all 8 MCS at ragged lengths, truncated and
 * corrupt inputs, every Viterbi depth and call granularity, the threaded batch paths), so
 * that an out-of-bounds access, a use of freed memory or undefined arithmetic in the checker
 * shows up here rather than as a silent parity difference.  Exit status 0 = all checks held.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "ziria_oracle.h"

static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { fails++; fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
                                        fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); } } while (0)

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return (uint32_t)rng; }

static const int MCS[8][2] = {{0, 0}, {0, 2}, {1, 0}, {1, 2}, {2, 0}, {2, 2}, {3, 1}, {3, 2}};
static const int NIBBLE[8] = {0xB, 0xF, 0xA, 0xE, 0x9, 0xD, 0x8, 0xC};   /* parsePLCPHeader.blk */

/* 24 header bits (rate, reserved, LENGTH, parity, tail) as 3 LSB-first bytes */
static void header_bytes(int m, int len, uint8_t* hb) {
  uint32_t h = (uint32_t)NIBBLE[m] | ((uint32_t)len << 5);
  h |= (uint32_t)(__builtin_popcount(h) & 1) << 17;
  hb[0] = h & 0xFF; hb[1] = (h >> 8) & 0xFF; hb[2] = (h >> 16) & 0xFF;
}

/* frequency-domain round trip: SIGNAL + data subcarriers -> rx_packet_freq */
static void freq_round_trip(int m, int plen, int drop) {
  const int mod = MCS[m][0], cod = MCS[m][1];
  uint8_t* pay = malloc(plen + 1);
  for (int i = 0; i < plen; i++) pay[i] = rnd();
  const int nd = zo_ndbps(mod, cod);
  const int nsym = (16 + 8 * plen + 32 + 6 + nd - 1) / nd;
  zo_c16* sub = malloc(sizeof(zo_c16) * 48 * (size_t)(1 + nsym));
  zo_tx_signal_symbol(mod, cod, plen + 4, sub);
  const int got = zo_tx_data_symbols(pay, plen, mod, cod, sub + 48, nsym);
  CHECK(got == nsym, "mcs %d len %d: %d data symbols, expected %d", m, plen, got, nsym);
  const int att = mod == 3 ? 110 : 80;               /* encdec_atten(16*5) (test_encdec.blk); 64-QAM */
  for (int i = 0; i < 48 * (1 + nsym); i++) {      /* needs its points inside DemapLimit's range */
    sub[i].re = (int16_t)(sub[i].re / att); sub[i].im = (int16_t)(sub[i].im / att);
  }
  uint8_t* out = calloc(4096, 1);
  zo_rx_result r;
  const int avail = 1 + nsym - drop;
  const int ret = zo_rx_packet_freq(sub, avail, out, &r);
  if (drop == 0) {
    CHECK(ret == 0 && r.crc_ok == 1, "mcs %d len %d: ret %d crc %d", m, plen, ret, r.crc_ok);
    CHECK(r.h.len == plen + 4 && r.h.modulation == mod && r.h.coding == cod, "mcs %d len %d header", m, plen);
    CHECK(memcmp(out, pay, plen) == 0, "mcs %d len %d payload", m, plen);
  } else {
    CHECK(ret < 0 || r.crc_ok != 1, "mcs %d len %d truncated by %d decoded", m, plen, drop);
  }
  free(out); free(sub); free(pay);
}

/* time-domain round trip through the whole transmitter and the stream receiver */
static void stream_round_trip(int m, int plen) {
  uint8_t* in = malloc(3 + plen);
  header_bytes(m, plen + 4, in);
  for (int i = 0; i < plen; i++) in[3 + i] = rnd();
  const int nd = zo_ndbps(MCS[m][0], MCS[m][1]);
  const int nsym = (16 + 8 * plen + 32 + 6 + nd - 1) / nd;
  const int pre = 1000;                             /* append_idle (test_tx loopback) */
  const int cap = pre + 640 + 160 * (1 + nsym) + 1024;
  zo_c16* x40 = calloc(cap, sizeof(zo_c16));
  const int n40 = zo_tx_packet(in, 3 + plen, x40 + pre, cap - pre - 512);
  CHECK(n40 > 0, "tx_packet mcs %d len %d -> %d", m, plen, n40);
  if (n40 <= 0) { free(in); free(x40); return; }
  const int total = ((pre + n40 + 512) / 8) * 8;
  for (int i = 0; i < total; i++) {                 /* amp(10), as the test_tx loopback */
    x40[i].re = (int16_t)(10 * x40[i].re);
    x40[i].im = (int16_t)(10 * x40[i].im);
  }
  zo_c16* x20 = malloc(sizeof(zo_c16) * (size_t)total / 2);
  const int n20 = zo_downsample(x40, total, x20);
  uint8_t* out = calloc(4096, 1);
  zo_rx_result r; zo_cca det; zo_c16 coeffs[64]; int d0 = 0;
  const int ret = zo_rx_stream(x20, n20, out, &r, &det, coeffs, &d0);
  /* the noiseless loopback decodes at BPSK/QPSK; the QAM rates exercise the same code
     (whether the LTS estimate of an unfaded x10 capture holds their points is not the
     question here) */
  if (MCS[m][0] <= 1)
    CHECK(ret == 0 && r.crc_ok == 1 && memcmp(out, in + 3, plen) == 0,
          "stream mcs %d len %d: ret %d crc %d", m, plen, ret, r.crc_ok);
  /* the same stream cut inside the data symbols */
  const int cut = d0 + 80 * (r.nsym_used > 2 ? r.nsym_used / 2 : 1);
  if (cut < n20) {
    memset(out, 0, 4096);
    const int ret2 = zo_rx_stream(x20, cut, out, &r, &det, coeffs, &d0);
    CHECK(ret2 != 0 || r.crc_ok != 1, "cut stream mcs %d len %d decoded", m, plen);
  }
  free(out); free(x20); free(x40); free(in);
}

/* A frame longer than the 40000-column trellis (frame_len 6000): the oracle and the port's
   batched brick stop consuming at the cap instead of reading and writing past it; both
   produce the same windows up to there. */
static void over_cap(void) {
  const int fl = 6000, n = 48 * 2100;                  /* 100800 soft values, rate 1/2: 50400 columns */
  int8_t* soft = malloc(n);
  for (int i = 0; i < n; i++) soft[i] = (int8_t)(rnd() & 7);
  zo_vit v; memset(&v, 0, sizeof(v));
  CHECK(zo_vit_init(&v, fl, 0, 256) == 0, "vit_init");
  uint8_t* a = calloc(fl + 64, 1);
  uint8_t* b = calloc(fl + 64, 1);
  const int got = zo_vit_decode(&v, soft, n, a);
  CHECK(got > 0 && got < 40000 && got % 256 == 0, "over-cap frame: %d bits", got);
  const int64_t off = 0, oo = 0;
  const int32_t sl = n, flen = fl;
  const int16_t cr = 0;
  zp_viterbi_batch(soft, &off, &sl, &flen, &cr, 1, b, &oo, 1);
  CHECK(memcmp(a, b, (size_t)got / 8) == 0, "over-cap frame: port differs from the oracle");
  zo_vit_free(&v);
  free(soft); free(a); free(b);
}

/* Viterbi brick: encoded random frames (zero-padded to whole 48-soft blocks, as the RX
   feeds it), fed whole, per 48-soft call and per 7 x 48 */
static void viterbi_calls(int cr, int fl, int depth) {
  const int K = cr == 0 ? 24 : cr == 1 ? 32 : 36;    /* data bits per 48 soft values */
  const int nbits = (8 * fl + 6 + K - 1) / K * K;
  uint8_t* bits = calloc(nbits + 64, 1);
  for (int i = 0; i < 8 * fl; i++) bits[i] = rnd() & 1;
  uint8_t* coded = calloc(4 * (size_t)nbits + 256, 1);
  const int ncoded = zo_tx_encode(bits, nbits, cr, coded);
  int8_t* soft = malloc((size_t)ncoded + 64);
  for (int i = 0; i < ncoded; i++) soft[i] = coded[i] ? 7 : 0;   /* hard decisions as soft */
  const int n = ncoded;
  uint8_t* first = NULL;
  int first_bits = 0;
  CHECK(n % 48 == 0, "cr %d fl %d: %d soft values", cr, fl, n);
  for (int mode = 0; mode < 3; mode++) {
    zo_vit v; memset(&v, 0, sizeof(v));
    CHECK(zo_vit_init(&v, fl, cr, depth) == 0, "vit_init");
    uint8_t* out = calloc((size_t)fl + 64, 1);
    int got = 0;
    const int step = mode == 0 ? n : mode == 1 ? 48 : 7 * 48;
    for (int a = 0; a < n; a += step) {
      const int k = a + step <= n ? step : n - a;
      got += zo_vit_decode(&v, soft + a, k, out + got / 8);
    }
    if (mode == 0) { first = malloc((size_t)fl + 64); memcpy(first, out, (size_t)fl + 64); first_bits = got; }
    else CHECK(got == first_bits && memcmp(first, out, (size_t)fl + 64) == 0,
               "cr %d fl %d depth %d: mode %d differs from one call", cr, fl, depth, mode);
    if (depth >= 24) {             /* depth 1 is honoured as the brick does, not a useful decoder */
      CHECK(got >= 8 * fl, "cr %d fl %d depth %d mode %d: %d bits", cr, fl, depth, mode, got);
      int ok = 1;
      for (int i = 0; i < 8 * fl && ok; i++) ok = ((out[i / 8] >> (i % 8)) & 1) == bits[i];
      CHECK(ok, "cr %d fl %d depth %d mode %d: wrong bits", cr, fl, depth, mode);
    }
    zo_vit_free(&v);
    free(out);
  }
  free(first); free(soft); free(coded); free(bits);
}

/* batched paths on worker threads (the bench's cpu_baseline leg) */
static void batches(void) {
  enum { N = 24 };
  int64_t off[N]; int32_t ns[N]; int lens[N], mcs[N];
  int64_t total = 0;
  for (int p = 0; p < N; p++) {
    mcs[p] = p % 8; lens[p] = 1 + (int)(rnd() % 1600);
    const int nd = zo_ndbps(MCS[mcs[p]][0], MCS[mcs[p]][1]);
    ns[p] = 1 + (16 + 8 * lens[p] + 38 + nd - 1) / nd - (p == 5);   /* packet 5 truncated */
    off[p] = total; total += ns[p];
  }
  zo_c16* sub = calloc((size_t)total * 48, sizeof(zo_c16));
  zo_c16* sym = calloc((size_t)total * 64, sizeof(zo_c16));
  uint8_t** pays = malloc(sizeof(uint8_t*) * N);
  for (int p = 0; p < N; p++) {
    pays[p] = malloc(lens[p]);
    for (int i = 0; i < lens[p]; i++) pays[p][i] = rnd();
    const int mod = MCS[mcs[p]][0], cod = MCS[mcs[p]][1];
    zo_tx_signal_symbol(mod, cod, lens[p] + 4, sub + 48 * off[p]);
    const int nd = zo_ndbps(mod, cod);
    const int full = (16 + 8 * lens[p] + 38 + nd - 1) / nd;
    zo_c16* tmp = malloc(sizeof(zo_c16) * 48 * (size_t)full);
    zo_tx_data_symbols(pays[p], lens[p], mod, cod, tmp, full);
    memcpy(sub + 48 * (off[p] + 1), tmp, sizeof(zo_c16) * 48 * (size_t)(ns[p] - 1));
    free(tmp);
    for (int k = 0; k < ns[p]; k++) {               /* subcarriers -> time domain (k: pilot index) */
      zo_c16 f[64], t[64];
      memset(f, 0, sizeof(f));
      static const int data_bins[48] = {38, 39, 40, 41, 42, 44, 45, 46, 47, 48, 49, 50, 51, 52, 53, 54, 55, 56,
                                        58, 59, 60, 61, 62, 63, 1, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 13, 14,
                                        15, 16, 17, 18, 19, 20, 22, 23, 24, 25, 26};
      for (int i = 0; i < 48; i++) f[data_bins[i]] = sub[48 * (off[p] + k) + i];
      zo_ifft64(f, t);
      memcpy(sym + 64 * (off[p] + k), t, sizeof(t));
    }
  }
  uint8_t* pay = calloc((size_t)N * 4096, 1);
  zo_rx_result res[N];
  CHECK(zo_rx_batch_time(sym, off, ns, N, pay, 4096, res, 4) == 0, "rx_batch_time");
  /* the frequency-domain path is the checked one here; the time path must agree with it
     packet for packet (same chain after the FFT) */
  for (int p = 0; p < N; p++) {
    uint8_t* one = calloc(4096, 1);
    zo_rx_result r1;
    zo_rx_packet_time(sym + 64 * off[p], ns[p], one, &r1);
    CHECK(r1.crc_ok == res[p].crc_ok && memcmp(one, pay + 4096 * (size_t)p, 4096) == 0, "batch vs single %d", p);
    free(one);
  }
  {                                                  /* the fast CPU port (bench's baseline) */
    uint8_t* payp = calloc((size_t)N * 4096, 1);
    zo_rx_result resp[N];
    zp_rx_batch_time(sym, off, ns, N, payp, 4096, resp, 3);
    for (int p = 0; p < N; p++)
      CHECK(resp[p].crc_ok == res[p].crc_ok && resp[p].h.len == res[p].h.len &&
            memcmp(payp + 4096 * (size_t)p, pay + 4096 * (size_t)p, 4096) == 0, "port vs oracle %d", p);
    free(payp);
  }
  zo_c16 chan[N * 64];
  for (int i = 0; i < N * 64; i++) { chan[i].re = 256; chan[i].im = 0; }   /* unit taps (>> 8) */
  uint8_t* pay2 = calloc((size_t)N * 4096, 1);
  zo_rx_result res2[N];
  CHECK(zo_rx_batch_time_eq(sym, off, ns, N, chan, pay2, 4096, res2, 3) == 0, "rx_batch_time_eq");
  /* Viterbi batch on the soft values of synthetic frames, 5 threads */
  enum { V = 10 };
  int64_t soff[V + 1], oo[V]; int32_t sl[V], fl[V]; int16_t crs[V];
  int64_t st = 0, ot = 0;
  for (int p = 0; p < V; p++) {
    crs[p] = p % 3; fl[p] = 1 + (int)(rnd() % 700);
    const int grp = crs[p] == 0 ? 2 : crs[p] == 1 ? 3 : 4;
    sl[p] = ((16 * fl[p] + 12) * (crs[p] == 0 ? 2 : crs[p] == 1 ? 3 : 4) / (crs[p] == 0 ? 1 : crs[p] == 1 ? 2 : 3) / grp) * grp;
    soff[p] = st; st += sl[p]; oo[p] = ot; ot += fl[p] + 64;
  }
  int8_t* soft = malloc((size_t)st + 64);
  for (int64_t i = 0; i < st; i++) soft[i] = (int8_t)(rnd() % 8);
  uint8_t* vout = calloc((size_t)ot, 1);
  zo_viterbi_batch(soft, soff, sl, fl, crs, V, vout, oo, 5);
  for (int p = 0; p < V; p++) {                      /* equal to the brick fed in one call */
    zo_vit v; memset(&v, 0, sizeof(v));
    zo_vit_init(&v, fl[p], crs[p], 256);
    uint8_t* one = calloc((size_t)fl[p] + 64, 1);
    zo_vit_decode(&v, soft + soff[p], sl[p], one);
    CHECK(memcmp(one, vout + oo[p], fl[p]) == 0, "viterbi batch %d", p);
    zo_vit_free(&v);
    free(one);
  }
  free(vout); free(soft); free(pay2); free(pay);
  for (int p = 0; p < N; p++) free(pays[p]);
  free(pays); free(sym); free(sub);
}

int main(void) {
  const int lens[] = {1, 2, 17, 100, 1500, 2044};
  for (int m = 0; m < 8; m++)
    for (unsigned i = 0; i < sizeof(lens) / sizeof(lens[0]); i++) {
      freq_round_trip(m, lens[i], 0);
      freq_round_trip(m, lens[i], 1);
    }
  for (int m = 0; m < 8; m++) stream_round_trip(m, 300);
  for (int m = 0; m < 8; m++) stream_round_trip(m, 40 + 97 * m);
  stream_round_trip(0, 700);
  const int depths[] = {1, 24, 64, 256, 1000};
  for (int cr = 0; cr < 3; cr++)
    for (unsigned d = 0; d < sizeof(depths) / sizeof(depths[0]); d++) viterbi_calls(cr, 1 + 37 * cr + 100 * d, depths[d]);
  batches();
  over_cap();
  /* corrupt SIGNAL: random bits in every header field, no packet behind it */
  for (int t = 0; t < 64; t++) {
    zo_c16 sub[48 * 4];
    for (int i = 0; i < 48 * 4; i++) { sub[i].re = (int16_t)rnd(); sub[i].im = (int16_t)rnd(); }
    uint8_t* out = calloc(4096, 1);
    zo_rx_result r;
    zo_rx_packet_freq(sub, 4, out, &r);
    free(out);
  }
  printf("asan_selftest: %s (%d failures)\n", fails ? "FAILED" : "ok", fails);
  return fails ? 1 : 0;
}
