// Test-infrastructure only.  Wraps the reference Viterbi brick
// (/root/reference/csrc/sora_ext_viterbi.cpp, compiled from where it lies) under zref_*
// names.  Built into oracle/_ref/ only.
#include <stdint.h>
#include <string.h>
#include "sora_ext_viterbi.cpp"
extern "C" __attribute__((visibility("default")))
int zref_viterbi_init(int frame_len, int code_rate, int depth) {
  return __ext_viterbi_brick_init_fast(frame_len, (int16)code_rate, (int16)depth);
}
extern "C" __attribute__((visibility("default")))
int zref_viterbi_decode(signed char* soft, int n, unsigned char* bits, int bits_len) {
  return __ext_viterbi_brick_decode_fast((num8*)soft, n, bits, bits_len);
}
extern "C" __attribute__((visibility("default")))
int zref_viterbi_sig(signed char* soft48, unsigned char* bits4) {
  return __ext_viterbiSig11a_brick_decode_fast((num8*)soft48, 48, bits4, 32);
}
// Copies of the brick's branch-metric LUTs (viterbilut.h) for a direct table check.
extern "C" __attribute__((visibility("default")))
void zref_viterbi_luts(unsigned char* ma1024, unsigned char* mb1024) {
  memcpy(ma1024, (const void*)VIT_MA, 1024);
  memcpy(mb1024, (const void*)VIT_MB, 1024);
}
