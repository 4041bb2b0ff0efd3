# tsan.mk -- host code of the device paths under ThreadSanitizer, built beside the product (the
# kernel build recipe in ../../Makefile is part of the counter stamps' source hash; this is not):
#   make -f tests/cpp/tsan.mk        (from the repository root; __graft_entry__.build() runs it)
# ROCm's clang++: gcc 11's TSAN misreports condition_variable::wait_for. Host instrumentation
# only (no GPU sanitizer); tests/test_sanitizers.py runs the binaries on the GPU with the ROCm
# runtime suppressed (tests/tsan_rocm.supp).
# The programs link build/tsan/lib/libfi_learner.so: the product's device objects with the
# library's host side (csrc/learner.cpp: staging threads, async steps, communicator, errors)
# recompiled with host-only TSAN instrumentation, so its own threads are checked too.
CLANGXX ?= /opt/rocm/lib/llvm/bin/clang++
HIPCC ?= /opt/rocm/bin/hipcc
CSRC := freeimpala_amd/csrc
TLIB := build/tsan/lib
DEVOBJS := $(patsubst %,build/obj/%.hip.o,farmer vtrace gemm_f32 misc atari atari_fr fc_gemm)
TSAN_LINK := -pthread -L$(TLIB) -lfi_learner '-Wl,-rpath,$$ORIGIN/lib' -Wl,-rpath,/opt/rocm/lib
HDRS := $(wildcard include/freeimpala_amd/*.hpp) include/fi_learner.h $(TLIB)/libfi_learner.so

all: build/tsan/host_learner_check build/tsan/fi_freeimpala asan

build/tsan/learner.cpp.o: $(CSRC)/learner.cpp $(wildcard $(CSRC)/*.h) include/fi_learner.h
	@mkdir -p build/tsan
	$(HIPCC) --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -Iinclude -I$(CSRC) -Wno-unused-value -Wno-unused-result -Xarch_host -fsanitize=thread -x hip -c $< -o $@

$(TLIB)/libfi_learner.so: build/tsan/learner.cpp.o $(DEVOBJS)
	@mkdir -p $(TLIB)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

build/tsan/host_learner_check: tests/cpp/host_learner_check.cpp $(HDRS)
	@mkdir -p build/tsan
	$(CLANGXX) -std=c++17 -O1 -g -fsanitize=thread -Iinclude $< -o $@ $(TSAN_LINK)

build/tsan/fi_freeimpala: tools/fi_freeimpala.cpp tools/cli_common.hpp $(HDRS)
	@mkdir -p build/tsan
	$(CLANGXX) -std=c++17 -O1 -g -fsanitize=thread -Iinclude $< -o $@ $(TSAN_LINK)

# The same two programs and the library's host side under AddressSanitizer + UBSan (host-only
# instrumentation again; tests/test_sanitizers.py runs them on the GPU with leak checking off,
# since the ROCm runtime keeps its allocations to process exit).
ALIB := build/asan/lib
ASAN_LINK := -pthread -L$(ALIB) -lfi_learner '-Wl,-rpath,$$ORIGIN/lib' -Wl,-rpath,/opt/rocm/lib
AHDRS := $(wildcard include/freeimpala_amd/*.hpp) include/fi_learner.h $(ALIB)/libfi_learner.so

asan: build/asan/host_learner_check build/asan/fi_freeimpala

build/asan/learner.cpp.o: $(CSRC)/learner.cpp $(wildcard $(CSRC)/*.h) include/fi_learner.h
	@mkdir -p build/asan
	$(HIPCC) --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -Iinclude -I$(CSRC) -Wno-unused-value -Wno-unused-result -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all -x hip -c $< -o $@

$(ALIB)/libfi_learner.so: build/asan/learner.cpp.o $(DEVOBJS)
	@mkdir -p $(ALIB)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

build/asan/host_learner_check: tests/cpp/host_learner_check.cpp $(AHDRS)
	@mkdir -p build/asan
	$(CLANGXX) -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all -Iinclude $< -o $@ $(ASAN_LINK)

build/asan/fi_freeimpala: tools/fi_freeimpala.cpp tools/cli_common.hpp $(AHDRS)
	@mkdir -p build/asan
	$(CLANGXX) -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all -Iinclude $< -o $@ $(ASAN_LINK)
