# Host-side sanitizer build (SURVEY.md §5 "Race detection / sanitizers").
#   make asan       oracle self-test under ASan+UBSan, plus the C-ABI library's host half and
#                   the batching driver built with -fsanitize=address,undefined (device code
#                   unchanged: GPU sanitizers are not available on this pool), the driver's
#                   CPU tests run through it, and the per-call externals (host path) exercised
#                   by percall_bench.  Log: profiles/<round>_asan.log
#   make asan-gpu   (on a GPU box, after `make asan-build`) the driver's GPU tests (receiver
#                   KATs, packet manifest) through the sanitized host code.
ASAN_DIR := ziria_amd/_lib/asan
HOST_SAN := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer
SAN_ENV  := ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
CSRC     := $(wildcard ziria_amd/csrc/*.hip ziria_amd/csrc/*.hpp ziria_amd/csrc/*.h ziria_amd/csrc/*.cpp) include/ziria_rx.h
CLANG    := /opt/rocm/llvm/bin/clang++

.PHONY: asan asan-build asan-oracle asan-gpu
asan: asan-oracle asan-build
	$(SAN_ENV) ZRX_DRIVER=$(ASAN_DIR)/ziria_rx_driver python -m pytest tests/test_driver.py -q -m "not gpu" -p no:cacheprovider
	$(SAN_ENV) $(ASAN_DIR)/ziria_rx_driver --input-file-name=/dev/null --input-file-mode=bin \
	  --output-file-name=/dev/null --output-file-mode=bin --batch-mode=packets --batch-manifest=/dev/null; \
	  rc=$$?; echo "driver without a GPU: exit $$rc"; test $$rc -ne 134 -a $$rc -ne 139
	$(SAN_ENV) $(ASAN_DIR)/percall_bench 3 1500

asan-oracle:
	$(MAKE) -C oracle asan

asan-build: $(ASAN_DIR)/libziria_rx.so $(ASAN_DIR)/ziria_rx_driver $(ASAN_DIR)/percall_bench

$(ASAN_DIR)/libziria_rx.so: $(CSRC)
	mkdir -p $(ASAN_DIR)
	for f in zrx_host zrx_ext_cxx; do $(CLANG) -O1 -g -std=c++17 -fPIC -fsanitize=address,undefined \
	  -fno-omit-frame-pointer -c ziria_amd/csrc/$$f.cpp -o $(ASAN_DIR)/$$f.o || exit 1; done
	cd ziria_amd/csrc && hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -pthread -Wall $(HOST_SAN) \
	  -o ../_lib/asan/libziria_rx.so zrx_api.hip -x none ../_lib/asan/zrx_host.o ../_lib/asan/zrx_ext_cxx.o

$(ASAN_DIR)/ziria_rx_driver: tools/ziria_rx_driver.cpp integration/csrc/hip_ext_batch.cpp $(ASAN_DIR)/libziria_rx.so
	$(CLANG) -O1 -g -std=c++17 -Wall -Iinclude -fsanitize=address,undefined -fno-omit-frame-pointer \
	  -o $@ tools/ziria_rx_driver.cpp integration/csrc/hip_ext_batch.cpp -L$(ASAN_DIR) -lziria_rx -Wl,-rpath,'$$ORIGIN'

# the host per-call externals (zrx_host.cpp: AVX2 Viterbi, plan FFT of every size) under ASan+UBSan
$(ASAN_DIR)/percall_bench: tools/percall_bench.cpp $(ASAN_DIR)/libziria_rx.so
	$(CLANG) -O1 -g -std=c++17 -Wall -Iinclude -fsanitize=address,undefined -fno-omit-frame-pointer \
	  -o $@ tools/percall_bench.cpp -L$(ASAN_DIR) -lziria_rx -Wl,-rpath,'$$ORIGIN'

asan-gpu: asan-build
	$(SAN_ENV) ZRX_DRIVER=$(ASAN_DIR)/ziria_rx_driver python -u -m pytest tests/test_driver.py -v -m gpu \
	  -p no:cacheprovider --timeout 120 --timeout-method thread
