// A stand-in for a wplc-compiled program (test infrastructure): it declares the externals
// exactly as wplc's code generator writes them into test.cpp and calls them, so building it
// with the reference's toolchain settings (g++ -std=c++11, csrc/Makefile:36,92-96) and
// linking it against libziria_rx.so proves the library resolves the symbols a real Ziria
// program references.  Nothing here includes include/ziria_rx.h.
//
// Types as generated code sees them through "types.h": num8 = char, num16 = short, num32 =
// int (csrc/numerics.h:64-69), int8/int16/int32 = num8/num16/num32 (csrc/types.h:28-33),
// BitArrPtr = unsigned char* (csrc/bit.h:22), complex16 (csrc/numerics.h:113-116).
// Prototypes as cgFunExternal emits them (src/Codegen/CgFun.hs:287-316): array arguments
// become (T* name, int len) (cg_array_param, :108-116), an array result comes first
// (cgParamsByRef of __retf_<name>), a unit result is int (CgTypes.hs unitTy), and bit arrays
// are BitArrPtr (codeGenArrTyPtrOcc_).  Declarations from lib/externals.blk:110,201-217 and
// the batched externals of INTEGRATION.md §2.
//
//   wplc_caller viterbi <soft.bin> <frame_len> <code_rate> <out.bin>   per call, 48 soft values each
//   wplc_caller sig <soft48.bin> <out.bin>
//   wplc_caller fft <in.bin> <N> <out.bin>                             one transform of N points
//   wplc_caller shift <in.bin> <shift> <out.bin>                       v_shift_right_complex16
//   wplc_caller vbatch <soft.bin> <frame_len> <code_rate> <out.bin>    one-packet batch (GPU)
//   wplc_caller rx <sym.bin> <manifest> <payload.bin> <info.bin>       __ext_wifi_rx_batch (GPU)
//   wplc_caller rxstatic <sym.bin> <manifest> <payload.bin> <info.bin> <log.txt>
//       the same from arrays in static storage, as wplc emits a program's arrays: three calls
//       on the same arrays, the third after packet 5's SIGNAL symbol was wiped (GPU)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef char num8;
typedef short num16;
typedef int num32;
typedef num8 int8;
typedef num16 int16;
typedef num32 int32;
typedef unsigned char* BitArrPtr;
typedef struct complex16 { num16 re; num16 im; } complex16;

void __ext_sora_fft(complex16* __retf_sora_fft, int __len_unused_1, complex16* inp, int __len_unused_2);
void __ext_sora_fft_dynamic(complex16* __retf_sora_fft_dynamic, int __len_unused_3, int16 nFFTSize, complex16* inp,
                            int __len_unused_4);
int __ext_viterbi_brick_init_fast(int32 frame_length, int16 code_rate, int16 depth);
int16 __ext_viterbi_brick_decode_fast(int8* svalue, int __len_unused_5, BitArrPtr bitValue, int __len_unused_6);
int __ext_viterbiSig11a_brick_init_fast(int32 frame_length, int16 code_rate, int16 depth);
int16 __ext_viterbiSig11a_brick_decode_fast(int8* svalue, int __len_unused_7, BitArrPtr bitValue, int __len_unused_8);
int __ext_v_shift_right_complex16(complex16* z, int __len_unused_9, complex16* x, int __len_unused_10, int32 shift);
int32 __ext_viterbi_batch_decode(int8* soft, int __len_unused_11, int32* pkt_soft_off, int __len_unused_12,
                                 int32* frame_len, int __len_unused_13, int16* code_rate, int __len_unused_14,
                                 BitArrPtr out, int __len_unused_15, int32* pkt_out_off, int __len_unused_16);
int32 __ext_wifi_rx_batch(complex16* sym, int __len_unused_17, int32* pkt_sym_off, int __len_unused_18,
                          BitArrPtr payload, int __len_unused_19, int32* pkt_info, int __len_unused_20);

extern "C" int zrx_node_stats(long long* stats8);   // (libziria_rx.so's node counters; test only)

// rxstatic's arrays: file-scope globals like the `calign` arrays of wplc's generated code
static complex16 g_sym[2048 * 57 * 64];
static unsigned char g_pay[2048 * 4096];
static int32 g_info[2048 * 8];
static int32 g_off[2049];

static std::vector<char> slurp(const char* name) {
  std::vector<char> v;
  FILE* f = std::fopen(name, "rb");
  if (!f) { std::perror(name); std::exit(2); }
  char buf[65536];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) v.insert(v.end(), buf, buf + n);
  std::fclose(f);
  return v;
}
static void spill(const char* name, const void* p, size_t n) {
  FILE* f = std::fopen(name, "wb");
  if (!f) { std::perror(name); std::exit(2); }
  if (n) std::fwrite(p, 1, n, f);
  std::fclose(f);
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const char* mode = argv[1];
  if (!std::strcmp(mode, "viterbi") && argc == 6) {
    std::vector<char> soft = slurp(argv[2]);
    std::vector<unsigned char> bits(96000 / 8 + 64);           // arr[96000] bit of Viterbi.blk
    __ext_viterbi_brick_init_fast(std::atoi(argv[3]), (int16)std::atoi(argv[4]), 256);
    size_t nbytes = 0;
    for (size_t k = 0; k + 48 <= soft.size(); k += 48) {
      const int16 nb = __ext_viterbi_brick_decode_fast(soft.data() + k, 48, bits.data() + nbytes, 96000);
      nbytes += nb / 8;
    }
    spill(argv[5], bits.data(), nbytes);
    return 0;
  }
  if (!std::strcmp(mode, "sig") && argc == 4) {
    std::vector<char> soft = slurp(argv[2]);
    unsigned char w[4] = {0, 0, 0, 0};
    __ext_viterbiSig11a_brick_init_fast(3, 0, 24);
    __ext_viterbiSig11a_brick_decode_fast(soft.data(), 48, w, 24);
    spill(argv[3], w, 4);
    return 0;
  }
  if (!std::strcmp(mode, "fft") && argc == 5) {
    std::vector<char> raw = slurp(argv[2]);
    const int n = std::atoi(argv[3]);
    std::vector<complex16> in(n), out(n), dyn(n);
    std::memcpy(in.data(), raw.data(), (size_t)n * sizeof(complex16));
    __ext_sora_fft(out.data(), n, in.data(), n);
    __ext_sora_fft_dynamic(dyn.data(), n, (int16)n, in.data(), n);
    if (std::memcmp(out.data(), dyn.data(), (size_t)n * sizeof(complex16))) return 3;
    spill(argv[4], out.data(), (size_t)n * sizeof(complex16));
    return 0;
  }
  if (!std::strcmp(mode, "shift") && argc == 5) {
    std::vector<char> raw = slurp(argv[2]);
    const int n = (int)(raw.size() / sizeof(complex16));
    std::vector<complex16> z((size_t)n + 1);
    __ext_v_shift_right_complex16(z.data(), n, (complex16*)raw.data(), n, (int32)std::atoi(argv[3]));
    spill(argv[4], z.data(), (size_t)n * sizeof(complex16));
    return 0;
  }
  if (!std::strcmp(mode, "vbatch") && argc == 6) {
    std::vector<char> soft = slurp(argv[2]);
    int32 off[2] = {0, (int32)(soft.size() / 48 * 48)}, fl = std::atoi(argv[3]), oo = 0;
    int16 cr = (int16)std::atoi(argv[4]);
    std::vector<unsigned char> out((size_t)fl + 16);
    const int32 rc = __ext_viterbi_batch_decode(soft.data(), (int)soft.size(), off, 2, &fl, 1, &cr, 1, out.data(),
                                                (int)out.size() * 8, &oo, 1);
    if (rc != 1) { std::fprintf(stderr, "__ext_viterbi_batch_decode: %d\n", rc); return 1; }
    spill(argv[5], out.data(), (size_t)fl);
    return 0;
  }
  if (!std::strcmp(mode, "rx") && argc == 6) {
    std::vector<char> raw = slurp(argv[2]);
    std::vector<int32> off;
    FILE* m = std::fopen(argv[3], "r");
    if (!m) return 2;
    long v;
    while (std::fscanf(m, "%ld", &v) == 1) off.push_back((int32)v);
    std::fclose(m);
    const int np = (int)off.size() - 1;
    std::vector<unsigned char> pay((size_t)np * 4096);
    std::vector<int32> info((size_t)np * 8);
    const int32 rc = __ext_wifi_rx_batch((complex16*)raw.data(), (int)(raw.size() / 256), off.data(), (int)off.size(),
                                         pay.data(), (int)pay.size() * 8, info.data(), (int)info.size());
    if (rc < 0) { std::fprintf(stderr, "__ext_wifi_rx_batch: %d\n", rc); return 1; }
    spill(argv[4], pay.data(), pay.size());
    spill(argv[5], info.data(), info.size() * sizeof(int32));
    return 0;
  }
  if (!std::strcmp(mode, "rxstatic") && argc == 7) {
    std::vector<char> raw = slurp(argv[2]);
    FILE* m = std::fopen(argv[3], "r");
    if (!m) return 2;
    int n_off = 0;
    long v;
    while (n_off < 2049 && std::fscanf(m, "%ld", &v) == 1) g_off[n_off++] = (int32)v;
    std::fclose(m);
    const int np = n_off - 1;
    if (np < 6 || raw.size() > sizeof(g_sym) || (size_t)g_off[np] * 256 != raw.size()) return 2;
    std::memcpy(g_sym, raw.data(), raw.size());
    FILE* log = std::fopen(argv[6], "w");
    if (!log) return 2;
    int32 rc[3];
    for (int k = 0; k < 3; k++) {
      if (k == 2) std::memset(g_sym + (size_t)g_off[5] * 64, 0, 256);   // packet 5: SIGNAL symbol wiped
      const auto t0 = std::chrono::steady_clock::now();
      rc[k] = __ext_wifi_rx_batch(g_sym, g_off[np], g_off, n_off, g_pay, (int)sizeof(g_pay) * 8, g_info,
                                  (int)(sizeof(g_info) / sizeof(int32)));
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      long long st[8];
      zrx_node_stats(st);
      std::fprintf(log, "call %d rc %d ms %.3f stats", k, rc[k], ms);
      for (long long x : st) std::fprintf(log, " %lld", x);
      std::fprintf(log, " crc5 %d\n", g_info[8 * 5 + 4]);
      if (k == 1) spill(argv[4], g_pay, (size_t)np * 4096);
    }
    spill(argv[5], g_info, (size_t)np * 8 * sizeof(int32));
    std::fclose(log);
    return rc[0] < 0 || rc[1] < 0 || rc[2] < 0 ? 1 : 0;
  }
  return 2;
}
