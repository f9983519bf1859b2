// hip_ext_batch.cpp — the batching hook of the reference runtime's driver (north_star:
// "a batching hook in driver.cpp").  Drop this file into the
// reference's csrc/, apply driver.cpp.patch (next to this file) and link libziria_rx.so:
//
//   make -C csrc EXTRACOPTS="-DZIRIA_HIP_BATCH -I$ZIRIA_AMD/include"
//        OBJ_EXT="ext_math.o ext_arr.o hip_ext_batch.o"
//        LIBS="-lm -L$ZIRIA_AMD/ziria_amd/_lib -lziria_rx -Wl,-rpath,$ZIRIA_AMD/ziria_amd/_lib"
//
// (sora_ext_viterbi.o leaves the link: the library exports its externals.)  The reference's
// main (csrc/driver.cpp:146-338) runs one synchronous wpl_go() stream, which cannot batch.
// The patched main first calls hip_ext_batch_main(argc, argv): without --batch-mode it
// returns -1 and the program runs exactly as before (wplc's state machine, the per-call
// externals); with it, the whole input file is decoded by one batched call and main returns
// its exit code.
//
// Flags (the reference's own file flags, csrc/params.c:215-226, plus the batch ones):
//   --input-file-name=F --input-file-mode=dbg|bin     int16 samples (re, im interleaved):
//                                                      dbg = comma-separated decimal text
//                                                      (buf_numerics16.c:45-83), bin = raw int16
//   --output-file-name=F --output-file-mode=dbg|bin   payload bytes as int8 (buf_numerics8.c:
//                                                      dbg "%d" then ",%d"; bin raw bytes)
//   --batch-mode=receiver  receiver() (receiver.blk:57-72) once per capture
//                          (__ext_wifi_rx_stream_batch); --batch-manifest=M lists captures as
//                          "first_sample nsamples" lines (default: the whole file is one
//                          capture); --batch-idle=N prepends N zero samples and
//                          --batch-scale=K multiplies the samples by K (the append_idle of
//                          code/WiFi/tests/test_*rx.blk); --batch-downsample applies downSample.blk
//   --batch-mode=packets   receiveBits after FFT/GetData on CP-removed symbols (64 complex16
//                          each, __ext_wifi_rx_batch); --batch-manifest=M lists packets as
//                          "first_symbol nsym" lines
//   --batch-mode=dry-run   parse the input and write it back as int16 in the output mode
//   --batch-max-bytes=N    write at most N payload bytes per packet (print_hdr of test_real_rx.blk)
//   --batch-info-file=F    per-packet "modulation,coding,len,header_err,crc_ok,status" lines
// The other flags of the reference's table (--input=, --heap-size=, ...) are accepted and
// ignored in batch mode.
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ziria_rx.h"

namespace {

struct Args {
  std::string in, out, in_mode = "bin", out_mode = "bin", mode, manifest, info;
  int idle = 0, scale = 1, max_bytes = -1;
  bool downsample = false;
};

bool starts(const char* a, const char* p, std::string* v) {
  const size_t n = std::strlen(p);
  if (std::strncmp(a, p, n) != 0) return false;
  if (v) *v = a + n;
  return true;
}

// flags of the reference's parameter table (csrc/params.c:190-330) batch mode ignores
const char* const kRefFlags[] = {"--DEBUG=", "--input=", "--output=", "--output-buffer-size=", "--dummy-samples=",
                                 "--heap-size=", "--input-file-repeat=", "--latency-sampling=",
                                 "--latency-sampling-location=", "--latency-CDF-size=", "--sdr-"};

int usage() {
  std::fprintf(stderr, "batch mode: --batch-mode=receiver|packets|dry-run --input-file-name=F "
                       "[--input-file-mode=dbg|bin] --output-file-name=F [--output-file-mode=dbg|bin] "
                       "[--batch-manifest=M] [--batch-idle=N] [--batch-scale=K] [--batch-downsample] "
                       "[--batch-max-bytes=N] [--batch-info-file=F]\n");
  return 2;
}

bool read_file(const std::string& name, std::string* data) {
  FILE* f = std::fopen(name.c_str(), "rb");
  if (!f) return false;
  char buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) data->append(buf, n);
  std::fclose(f);
  return true;
}

// parse_dbg_int16 (buf_numerics16.c:45-83): comma-separated integers, newlines count as
// separators as well (the reference's files put one vector per line)
bool parse_dbg(const std::string& text, std::vector<int16_t>* v) {
  const char* p = text.c_str();
  while (*p) {
    while (*p == ',' || *p == '\n' || *p == '\r' || *p == ' ' || *p == '\t') p++;
    if (!*p) break;
    char* end = nullptr;
    errno = 0;
    const long x = std::strtol(p, &end, 10);
    if (end == p || errno == EINVAL) return false;
    v->push_back((int16_t)x);
    p = end;
  }
  return true;
}

bool read_samples(const Args& a, std::vector<int16_t>* v) {
  std::string data;
  if (!read_file(a.in, &data)) return false;
  if (a.in_mode == "dbg") return parse_dbg(data, v);
  v->resize(data.size() / 2);
  if (!v->empty()) std::memcpy(v->data(), data.data(), v->size() * 2);
  return true;
}

bool read_manifest(const std::string& name, std::vector<int32_t>* first, std::vector<int32_t>* count) {
  FILE* f = std::fopen(name.c_str(), "r");
  if (!f) return false;
  long s, n;
  while (std::fscanf(f, "%ld %ld", &s, &n) == 2) {
    first->push_back((int32_t)s);
    count->push_back((int32_t)n);
  }
  std::fclose(f);
  return true;
}

struct Writer {
  FILE* f;
  bool dbg, any;
  Writer(FILE* f_, bool dbg_) : f(f_), dbg(dbg_), any(false) {}
  void put(int8_t x) {                              // buf_numerics8.c: "%d" then ",%d"
    if (dbg) {
      std::fprintf(f, any ? ",%d" : "%d", (int)x);
      any = true;
    } else {
      std::fputc((unsigned char)x, f);
    }
  }
  void put16(int16_t x) {                           // buf_numerics16.c:350-357, fwrite for bin
    if (dbg) {
      std::fprintf(f, any ? ",%d" : "%d", (int)x);
      any = true;
    } else {
      std::fwrite(&x, 2, 1, f);
    }
  }
};

}  // namespace

int hip_ext_batch_main(int argc, char** argv) {
  Args a;
  bool batch = false;
  for (int i = 1; i < argc; i++)
    if (starts(argv[i], "--batch-mode=", &a.mode)) batch = true;
  if (!batch) return -1;                             // not ours: the reference's main runs as before
  for (int i = 1; i < argc; i++) {
    std::string v;
    const char* s = argv[i];
    if (starts(s, "--batch-mode=", nullptr)) continue;
    else if (starts(s, "--input-file-name=", &v)) a.in = v;
    else if (starts(s, "--input-file-mode=", &v)) a.in_mode = v;
    else if (starts(s, "--output-file-name=", &v)) a.out = v;
    else if (starts(s, "--output-file-mode=", &v)) a.out_mode = v;
    else if (starts(s, "--batch-manifest=", &v)) a.manifest = v;
    else if (starts(s, "--batch-info-file=", &v)) a.info = v;
    else if (starts(s, "--batch-idle=", &v)) a.idle = std::atoi(v.c_str());
    else if (starts(s, "--batch-scale=", &v)) a.scale = std::atoi(v.c_str());
    else if (starts(s, "--batch-max-bytes=", &v)) a.max_bytes = std::atoi(v.c_str());
    else if (!std::strcmp(s, "--batch-downsample")) a.downsample = true;
    else {
      bool ref = false;
      for (const char* f : kRefFlags) ref |= starts(s, f, nullptr);
      if (!ref) return usage();
    }
  }
  if (a.in.empty() || a.out.empty() || (a.in_mode != "dbg" && a.in_mode != "bin") ||
      (a.out_mode != "dbg" && a.out_mode != "bin") ||
      (a.mode != "receiver" && a.mode != "packets" && a.mode != "dry-run"))
    return usage();
  std::vector<int16_t> raw;
  if (!read_samples(a, &raw)) {
    std::fprintf(stderr, "batch mode: cannot read %s\n", a.in.c_str());
    return 1;
  }
  FILE* out = std::fopen(a.out.c_str(), "wb");
  if (!out) {
    std::fprintf(stderr, "batch mode: cannot write %s\n", a.out.c_str());
    return 1;
  }
  Writer w(out, a.out_mode == "dbg");
  if (a.mode == "dry-run") {                         // int16 format round trip, no engine call
    for (int16_t x : raw) w.put16(x);
    std::fclose(out);
    return 0;
  }
  const int nsamp = (int)(raw.size() / 2);
  std::vector<int32_t> first, count;
  if (!a.manifest.empty()) {
    if (!read_manifest(a.manifest, &first, &count)) {
      std::fprintf(stderr, "batch mode: cannot read manifest %s\n", a.manifest.c_str());
      std::fclose(out);
      return 1;
    }
  } else {
    first.push_back(0);
    count.push_back(a.mode == "packets" ? nsamp / 64 : nsamp);
  }
  const int np = (int)first.size();
  std::vector<uint8_t> payload((size_t)np * 4096);
  std::vector<int32_t> info((size_t)np * 8);
  int32_t rc;
  if (a.mode == "receiver") {
    // each capture: idle zeros, then its samples times scale (append_idle), CSR offsets
    std::vector<int16_t> caps;
    std::vector<int32_t> off(1, 0);
    for (int i = 0; i < np; i++) {
      if (first[i] < 0 || count[i] < 0 || first[i] + (int64_t)count[i] > nsamp) { std::fclose(out); return usage(); }
      caps.insert(caps.end(), 2 * (size_t)a.idle, 0);
      for (int k = 0; k < 2 * count[i]; k++) caps.push_back((int16_t)(raw[2 * (size_t)first[i] + k] * a.scale));
      off.push_back((int32_t)(caps.size() / 2));
    }
    std::vector<int32_t> det((size_t)np * 8);
    rc = __ext_wifi_rx_stream_batch((complex16*)caps.data(), (int)(caps.size() / 2), off.data(), np + 1,
                                    a.downsample ? 1 : 0, payload.data(), (int)payload.size() * 8,
                                    info.data(), (int)info.size(), det.data(), (int)det.size());
    for (int i = 0; i < np && rc >= 0; i++)
      if (!det[8 * i]) info[8 * i + 4] = 0;         // no packet detected: nothing to emit
  } else {
    std::vector<int32_t> off(1, 0);
    std::vector<int16_t> syms;
    for (int i = 0; i < np; i++) {
      if (first[i] < 0 || count[i] < 0 || ((int64_t)first[i] + count[i]) * 64 > nsamp) { std::fclose(out); return usage(); }
      syms.insert(syms.end(), raw.begin() + 128 * (size_t)first[i], raw.begin() + 128 * (size_t)(first[i] + count[i]));
      off.push_back(off.back() + count[i]);
    }
    rc = __ext_wifi_rx_batch((complex16*)syms.data(), (int)(syms.size() / 128), off.data(), np + 1,
                             payload.data(), (int)payload.size() * 8, info.data(), (int)info.size());
  }
  if (rc < 0) {
    std::fprintf(stderr, "batch mode: engine error %d\n", rc);
    std::fclose(out);
    return 1;
  }
  FILE* inf = a.info.empty() ? nullptr : std::fopen(a.info.c_str(), "w");
  for (int i = 0; i < np; i++) {
    const int32_t* in = &info[8 * (size_t)i];
    if (inf) std::fprintf(inf, "%d,%d,%d,%d,%d,%d\n", in[0], in[1], in[2], in[3], in[4], in[5]);
    if (in[3] != 0 || in[5] != 0) continue;         // receiveBits emits nothing on a header error
    int nb = in[2] - 4;                               // CRC'd payload (crc(hdata.len-4), receiver.blk:47)
    if (a.max_bytes >= 0 && nb > a.max_bytes) nb = a.max_bytes;
    for (int k = 0; k < nb; k++) w.put((int8_t)payload[4096 * (size_t)i + k]);
  }
  if (inf) std::fclose(inf);
  std::fclose(out);
  return 0;
}
