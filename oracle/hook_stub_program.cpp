// Test infrastructure: a stand-in for the test.cpp wplc generates (src/Codegen/CgProgram.hs),
// providing the four entry points the reference's driver calls (csrc/driver.cpp:95-98,
// :229-230, :282, :296).  Its wpl_go() decodes nothing; it only lets the reference runtime
// link, so tests can run the patched driver's two paths: the unchanged stream path (this
// program) and the batching hook (integration/csrc/hip_ext_batch.cpp).
#include "types.h"

void wpl_global_init(memsize_int heap_size) { (void)heap_size; }
void wpl_input_initialize() {}
void wpl_output_finalize() {}
int wpl_go() { return 0; }
