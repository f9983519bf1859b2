// Standalone batching driver for libziria_rx.so: the batching hook of
// integration/csrc/hip_ext_batch.cpp as its own program, for callers without the reference
// runtime.  Same flags as the hook (--batch-mode=receiver|packets|dry-run plus the
// reference's --input-file-* / --output-file-* file flags); see that file.
#include <cstdio>

int hip_ext_batch_main(int argc, char** argv);

int main(int argc, char** argv) {
  const int rc = hip_ext_batch_main(argc, argv);
  if (rc < 0) {
    std::fprintf(stderr, "ziria_rx_driver: --batch-mode=receiver|packets|dry-run is required\n");
    return 2;
  }
  return rc;
}
