# Builds the product library (HIP for gfx950 + host C++) and the test oracle.
#   make            -> find-tfbs_amd/lib/libtfbs_amd.so, oracle/_build/libtfbs_oracle.so
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := find-tfbs_amd
SRC := $(PKG)/csrc
LIBDIR := $(PKG)/lib
OBJDIR := $(PKG)/lib/obj
JOBS ?= 8

HOST_SRCS := $(SRC)/patterns.cpp $(SRC)/plan.cpp $(SRC)/mfma.cpp $(SRC)/batch.cpp $(SRC)/aggregate.cpp $(SRC)/synth.cpp $(SRC)/io.cpp $(SRC)/inflate.cpp $(SRC)/run.cpp
HIP_SRCS := $(SRC)/device.hip $(SRC)/scan_kernels.hip $(SRC)/scan_mfma.hip $(SRC)/key_kernels.hip $(SRC)/bgzf_gpu.hip $(SRC)/build_gpu.hip
HDRS := $(wildcard $(SRC)/*.hpp) include/tfbs_amd.h
HOST_OBJS := $(patsubst $(SRC)/%.cpp,$(OBJDIR)/%.o,$(HOST_SRCS))
HIP_OBJS := $(patsubst $(SRC)/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS))

CXXFLAGS := -O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter
HIPFLAGS := $(CXXFLAGS) --offload-arch=$(ARCH) -munsafe-fp-atomics

all: $(LIBDIR)/libtfbs_amd.so $(PKG)/bin/find-tfbs-amd oracle

$(OBJDIR)/%.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(CXXFLAGS) -x c++ -c $< -o $@

# MFMA results straight into VGPRs (gfx950's unified register file): the
# threshold test reads every accumulator, so AGPR copies would cost 16 VALU per tile
$(OBJDIR)/scan_mfma.o: HIPFLAGS += -mllvm -amdgpu-mfma-vgpr-form -ffinite-math-only

$(OBJDIR)/%.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIBDIR)/libtfbs_amd.so: $(HOST_OBJS) $(HIP_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ -lz -lpthread

$(PKG)/bin/find-tfbs-amd: $(SRC)/cli.cpp include/tfbs_amd.h $(LIBDIR)/libtfbs_amd.so
	@mkdir -p $(PKG)/bin
	$(HIPCC) $(CXXFLAGS) -x c++ $< -o $@ -L$(LIBDIR) -ltfbs_amd -Wl,-rpath,'$$ORIGIN/../lib'

oracle:
	$(MAKE) -s -C oracle

asm: $(SRC)/scan_kernels.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip --cuda-device-only -S $< -o $(OBJDIR)/scan_kernels.s -Rpass-analysis=kernel-resource-usage

clean:
	rm -rf $(LIBDIR) $(PKG)/bin oracle/_build

.PHONY: all oracle clean asm
