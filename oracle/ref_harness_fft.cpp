// Test-infrastructure only (never shipped, never on the product path).
// Compiles the reference FFT brick from /root/reference/csrc (include path set by
// oracle/Makefile.ref) and exposes it under zref_* names so the oracle restatement
// can be checked against the real brick.  Built into oracle/_ref/ only.
#include "common.h"
extern "C" __attribute__((visibility("default")))
void zref_sora_fft(struct complex16* out, int n, struct complex16* in) {
  __ext_sora_fft(out, n, in, n);            // csrc/sora_ext_lib.cpp:2672
}
extern "C" __attribute__((visibility("default")))
int zref_v_shift_right_complex16(struct complex16* z, struct complex16* x, int len, int shift) {
  return __ext_v_shift_right_complex16(z, len, x, len, shift);   // csrc/sora_ext_lib.cpp:1979
}
