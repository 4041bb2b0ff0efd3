# tsan.mk -- host code of the device paths under ThreadSanitizer, built beside the product (the
# kernel build recipe in ../../Makefile is part of the counter stamps' source hash; this is not):
#   make -f tests/cpp/tsan.mk        (from the repository root; __graft_entry__.build() runs it)
# ROCm's clang++: gcc 11's TSAN misreports condition_variable::wait_for. Host instrumentation
# only (no GPU sanitizer); tests/test_sanitizers.py runs the binaries on the GPU with the ROCm
# runtime suppressed (tests/tsan_rocm.supp).
CLANGXX ?= /opt/rocm/lib/llvm/bin/clang++
LIBDIR := freeimpala_amd/lib
TSAN_LINK := -pthread -L$(LIBDIR) -lfi_learner '-Wl,-rpath,$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib
HDRS := $(wildcard include/freeimpala_amd/*.hpp) include/fi_learner.h $(LIBDIR)/libfi_learner.so

all: build/tsan/host_learner_check build/tsan/fi_freeimpala

build/tsan/host_learner_check: tests/cpp/host_learner_check.cpp $(HDRS)
	@mkdir -p build/tsan
	$(CLANGXX) -std=c++17 -O1 -g -fsanitize=thread -Iinclude $< -o $@ $(TSAN_LINK)

build/tsan/fi_freeimpala: tools/fi_freeimpala.cpp tools/cli_common.hpp $(HDRS)
	@mkdir -p build/tsan
	$(CLANGXX) -std=c++17 -O1 -g -fsanitize=thread -Iinclude $< -o $@ $(TSAN_LINK)
