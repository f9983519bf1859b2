// Per-call throughput of the drop-in externals on one host core: what a
// wplc-compiled RX that calls the bricks one OFDM symbol at a time (receiver/Decode.blk ->
// Viterbi, one __ext_viterbi_brick_decode_fast per symbol's soft values) gets from the
// library's host path (zrx_host.cpp), to set against the reference brick's 34-73 Mbit/s per
// core.  Includes this header as C++, so it calls the C++-linkage exports a
// wplc program links against.  Needs no GPU.
//
//   percall_bench [frames] [frame_len]
//
// For each code rate: init + one decode call per data symbol's soft values (48/96/192/288
// by modulation; here the rate's 802.11a partner modulation: 1/2 BPSK 48, 2/3 64-QAM 288,
// 3/4 64-QAM 288), `frames` frames of frame_len bytes, random soft values.  Also
// __ext_sora_fft per call at sizes 64, 12, 1200, 2048, 128.  Prints one JSON line.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../include/ziria_rx.h"

int main(int argc, char** argv) {
  const int frames = argc > 1 ? std::atoi(argv[1]) : 200;
  const int flen = argc > 2 ? std::atoi(argv[2]) : 1500;
  std::mt19937 rng(7);
  std::printf("{\"metric\": \"per-call externals on one host core\", \"frame_len\": %d, \"frames\": %d, \"viterbi\": [", flen,
              frames);
  const int per_call[3] = {48, 288, 288};
  const int bits_per_48[3] = {24, 32, 36};
  for (int cr = 0; cr < 3; cr++) {
    const int need = 8 * (flen + 2) + 6;
    const int blocks48 = (need + bits_per_48[cr] - 1) / bits_per_48[cr];
    const int pc = per_call[cr];
    const int nsoft = (blocks48 * 48 + pc - 1) / pc * pc;
    std::vector<char> soft(nsoft);
    for (auto& s : soft) s = (char)(rng() & 7);
    std::vector<uint8_t> out(flen + 4096);
    // one untimed frame (first call initialises the device)
    __ext_viterbi_brick_init_fast(flen + 2, (int16_t)cr, 256);
    for (int a = 0; a < nsoft; a += pc) __ext_viterbi_brick_decode_fast(soft.data() + a, pc, out.data(), (int)out.size());
    long calls = 0, bits = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int f = 0; f < frames; f++) {
      __ext_viterbi_brick_init_fast(flen + 2, (int16_t)cr, 256);
      int got = 0;
      for (int a = 0; a < nsoft; a += pc) {
        got += __ext_viterbi_brick_decode_fast(soft.data() + a, pc, out.data() + got / 8, (int)out.size() - got / 8);
        calls++;
      }
      bits += got;
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("%s{\"code_rate\": %d, \"soft_per_call\": %d, \"calls\": %ld, \"us_per_call\": %.2f, "
                "\"decoded_Mbit_s\": %.3f}", cr ? ", " : "", cr, pc, calls, s / calls * 1e6, bits / s / 1e6);
  }
  // __ext_sora_fft per call at a few of its sizes (the 802.11a symbol, the smallest and
  // largest LTE sizes, the largest power of two)
  std::printf("], \"sora_fft\": [");
  const int sizes[5] = {64, 12, 1200, 2048, 128};
  for (int si = 0; si < 5; si++) {
    const int N = sizes[si];
    std::vector<complex16> in(N), out(N);
    for (auto& c : in) { c.re = (int16_t)(rng() % 2001 - 1000); c.im = (int16_t)(rng() % 2001 - 1000); }
    __ext_sora_fft(out.data(), N, in.data(), 0);
    const int n = 20000;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) __ext_sora_fft(out.data(), N, in.data(), 0);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("%s{\"size\": %d, \"calls\": %d, \"us_per_call\": %.2f}", si ? ", " : "", N, n, s / n * 1e6);
  }
  std::printf("]}\n");
  return 0;
}
