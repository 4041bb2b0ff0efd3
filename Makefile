# Builds libfi_learner.so (HIP, gfx950 only) in-tree, plus the CPU oracle (test infra).
# No cmake needed; `python -c "import __graft_entry__ as g; g.build()"` drives the same rules.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := freeimpala_amd/csrc
LIBDIR := freeimpala_amd/lib
OBJDIR := build/obj
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Iinclude -I$(CSRC) -Wall -Wno-unused-result -Wno-unused-value \
            -munsafe-fp-atomics
SRCS := $(CSRC)/farmer.hip $(CSRC)/vtrace.hip $(CSRC)/gemm_f32.hip $(CSRC)/misc.hip $(CSRC)/atari.hip $(CSRC)/atari_fr.hip $(CSRC)/fc_gemm.hip $(CSRC)/learner.cpp
OBJS := $(patsubst $(CSRC)/%,$(OBJDIR)/%.o,$(SRCS))
HDRS := $(wildcard $(CSRC)/*.h) include/fi_learner.h include/fi_farmer.h

all: $(LIBDIR)/libfi_learner.so oracle host tools

$(OBJDIR)/%.hip.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.cpp.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIBDIR)/libfi_learner.so: $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -s -C oracle

# C++ host-side check program (include/freeimpala_amd/device_learner.hpp over the C ABI)
host: build/host_learner_check build/replay_check
build/replay_check: tests/cpp/replay_check.cpp $(wildcard include/freeimpala_amd/*.hpp) include/fi_learner.h $(LIBDIR)/libfi_learner.so
	@mkdir -p build
	g++ -std=c++17 -O2 -Wall -Wextra -Iinclude $< -o $@ -L$(LIBDIR) -lfi_learner -pthread '-Wl,-rpath,$$ORIGIN/../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib
build/host_learner_check: tests/cpp/host_learner_check.cpp include/freeimpala_amd/device_learner.hpp include/fi_learner.h $(LIBDIR)/libfi_learner.so
	@mkdir -p build
	g++ -std=c++17 -O2 -Wall -Iinclude $< -o $@ -L$(LIBDIR) -lfi_learner -pthread '-Wl,-rpath,$$ORIGIN/../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib

# the cmd/freeimpala-shaped binary on freeimpala_amd::Learner (include/freeimpala_amd/learner.hpp)
tools: build/fi_freeimpala build/fi_freeimpala_mpi
build/fi_freeimpala: tools/fi_freeimpala.cpp tools/cli_common.hpp $(wildcard include/freeimpala_amd/*.hpp) include/fi_learner.h $(LIBDIR)/libfi_learner.so
	@mkdir -p build
	g++ -std=c++17 -O2 -Wall -Wextra -Iinclude $< -o $@ -L$(LIBDIR) -lfi_learner -pthread '-Wl,-rpath,$$ORIGIN/../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib

# the freeimpala_mpi_async_pool-shaped binary (MPICH from /opt/conda; system libstdc++ first in
# the RPATH so conda's older copy is not picked up)
MPI_HOME ?= /opt/conda
MPI_LINK := $(MPI_HOME)/lib/libmpi.so -Wl,--disable-new-dtags -Wl,-rpath,/usr/lib/x86_64-linux-gnu:$(MPI_HOME)/lib
build/fi_freeimpala_mpi: tools/fi_freeimpala_mpi.cpp tools/cli_common.hpp $(wildcard include/freeimpala_amd/*.hpp) include/fi_learner.h $(LIBDIR)/libfi_learner.so
	@mkdir -p build
	g++ -std=c++17 -O2 -Wall -Wextra -Iinclude -I$(MPI_HOME)/include $< -o $@ -L$(LIBDIR) -lfi_learner -pthread '-Wl,-rpath,$$ORIGIN/../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib $(MPI_LINK)
build/mpi_pool_check: tests/cpp/mpi_pool_check.cpp $(wildcard include/freeimpala_amd/*.hpp)
	@mkdir -p build
	g++ -std=c++17 -O2 -Wall -Wextra -Iinclude -I$(MPI_HOME)/include $< -o $@ -pthread $(MPI_LINK)
host: build/mpi_pool_check

# INTEGRATION.md section 2's alias compiled on the reference's own classes (build container only:
# the reference tree is read in place, never copied; the binary travels to the GPU box)
REF ?= /root/reference
ifneq ($(wildcard $(REF)/include/freeimpala/data_structures.h),)
host: build/reference_binding build/reference_mpi_check
endif
build/reference_binding: tests/cpp/reference_binding.cpp tests/cpp/stubs/spdlog/spdlog.h $(wildcard include/freeimpala_amd/*.hpp) include/fi_learner.h $(LIBDIR)/libfi_learner.so
	@mkdir -p build
	g++ -std=c++17 -O2 -Wall -I$(REF)/include -Itests/cpp/stubs -Iinclude -include optional $< -o $@ -L$(LIBDIR) -lfi_learner -pthread '-Wl,-rpath,$$ORIGIN/../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib

# INTEGRATION.md section 3b's rank-0 patch (mpi::LearnerEndpoint) on the reference's own
# SharedBuffer / ModelManager, its Agent on the actor ranks, and the section 2 alias learner
build/reference_mpi_check: tests/cpp/reference_mpi_check.cpp tests/cpp/stubs/spdlog/spdlog.h $(wildcard include/freeimpala_amd/*.hpp) include/fi_learner.h $(LIBDIR)/libfi_learner.so
	@mkdir -p build
	g++ -std=c++17 -O2 -Wall -I$(REF)/include -Itests/cpp/stubs -Iinclude -I$(MPI_HOME)/include -include optional $< -o $@ -L$(LIBDIR) -lfi_learner -pthread '-Wl,-rpath,$$ORIGIN/../$(LIBDIR)' -Wl,-rpath,/opt/rocm/lib $(MPI_LINK)

clean:
	rm -rf build $(LIBDIR)
.PHONY: all oracle host tools clean
