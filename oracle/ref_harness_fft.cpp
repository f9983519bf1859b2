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
// Integer trigonometry and v_mul_complex16 of the reference (csrc/sora_ext_lib.cpp:2098,
// :2566-2580 over csrc/intalgx.h), for the ChannelEqualization / PilotTrack restatement.
extern "C" __attribute__((visibility("default")))
int zref_sin16(int r) { return __ext_sin_int16((int16)r); }
extern "C" __attribute__((visibility("default")))
int zref_cos16(int r) { return __ext_cos_int16((int16)r); }
extern "C" __attribute__((visibility("default")))
int zref_atan2_16(int y, int x) { return __ext_atan2_int16((int16)y, (int16)x); }
extern "C" __attribute__((visibility("default")))
void zref_v_mul_complex16(struct complex16* out, struct complex16* x, struct complex16* y, int len, int shift) {
  __ext_v_mul_complex16(out, len, x, len, y, len, shift);
}
// IFFT<64> brick (csrc/sora_ext_lib.cpp:2828), for the STS pattern of cca_tufv.blk
extern "C" __attribute__((visibility("default")))
void zref_sora_ifft64(struct complex16* out, struct complex16* in) { __ext_sora_ifft(out, 64, in, 64); }
extern "C" __attribute__((visibility("default")))
void zref_sora_ifft128(struct complex16* out, struct complex16* in) { __ext_sora_ifft(out, 128, in, 128); }
