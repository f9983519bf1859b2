// Test infrastructure: a stand-in for the test.cpp wplc generates (src/Codegen/CgProgram.hs),
// built the way a generated program is: it starts with cHeader's `#include "common.h"`
// (src/Codegen/CgHeader.hs:84), which pulls csrc/sora_ext_lib.cpp into the translation unit
// (csrc/common.h:24-25), and it declares the externals as cgFunExternal writes them
// (src/Codegen/CgFun.hs:287-316).  oracle/Makefile.hook compiles it with -DZIRIA_HIP_EXT
// against a scratch copy of sora_ext_lib.cpp patched by integration/csrc/sora_ext_lib.cpp.patch,
// so the program's __ext_sora_fft / __ext_sora_fft_dynamic / __ext_v_shift_right_complex16
// are undefined here and bind to libziria_rx.so.
//
// It provides the four entry points the reference's driver calls (csrc/driver.cpp:95-98,
// :229-230, :282, :296).  wpl_go() decodes nothing unless ZRX_STUB_FFT_IN names a file of
// complex16 blocks: then it runs __ext_sora_fft of ZRX_STUB_FFT_N points (default 64) on
// every block (and __ext_sora_fft_dynamic on the first) and writes ZRX_STUB_FFT_OUT, so a
// test can check which FFT the program bound and that it matches the reference KAT (the
// driver ignores wpl_go's result, so failures exit: 3 = file error, 4 = dynamic differs).
#include "common.h"

void __ext_sora_fft(complex16* __retf_sora_fft, int __len_unused_1, complex16* inp, int __len_unused_2);
void __ext_sora_fft_dynamic(complex16* __retf_sora_fft_dynamic, int __len_unused_3, int16 nFFTSize, complex16* inp,
                            int __len_unused_4);

void wpl_global_init(memsize_int heap_size) { (void)heap_size; }
void wpl_input_initialize() {}
void wpl_output_finalize() {}

int wpl_go() {
  const char* in = getenv("ZRX_STUB_FFT_IN");
  const char* out = getenv("ZRX_STUB_FFT_OUT");
  if (!in || !out) return 0;
  const int n = getenv("ZRX_STUB_FFT_N") ? atoi(getenv("ZRX_STUB_FFT_N")) : 64;
  FILE* f = fopen(in, "rb");
  if (!f || n <= 0) exit(3);
  fseek(f, 0, SEEK_END);
  const long blocks = ftell(f) / (long)(n * sizeof(complex16));
  fseek(f, 0, SEEK_SET);
  complex16* x = (complex16*)malloc(sizeof(complex16) * n * (blocks + 1));
  complex16* y = (complex16*)malloc(sizeof(complex16) * n * (blocks + 1));
  if (fread(x, sizeof(complex16) * n, blocks, f) != (size_t)blocks) exit(3);
  fclose(f);
  for (long b = 0; b < blocks; b++) __ext_sora_fft(y + b * n, n, x + b * n, n);
  if (blocks > 0) {          // the dynamic form of the first block must agree
    __ext_sora_fft_dynamic(y + blocks * n, n, (int16)n, x, n);
    if (memcmp(y + blocks * n, y, sizeof(complex16) * n) != 0) exit(4);
  }
  FILE* g = fopen(out, "wb");
  if (!g || fwrite(y, sizeof(complex16) * n, blocks, g) != (size_t)blocks) exit(3);
  fclose(g);
  free(x);
  free(y);
  return 0;
}
