# Top-level build: the gfx950 product library and the CPU oracle (test infra).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-inline-asm -fvisibility=hidden --offload-arch=$(ARCH) -Iinclude
LIBDIR := xsknf_amd/lib
LIB := $(LIBDIR)/libxsknf_gpu.so
SRCS := xsknf_amd/csrc/checksummer.hip xsknf_amd/csrc/host_path.hip

all: $(LIB) oracle

$(LIB): $(SRCS) include/xsknf_gpu.h xsknf_amd/csrc/checksummer_internal.h Makefile
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(SRCS)

# keep the device assembly for inspection (VGPRs, instruction mix)
asm: $(SRCS)
	@mkdir -p build/asm
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S -o build/asm/checksummer-gfx950.s xsknf_amd/csrc/checksummer.hip

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(LIBDIR) build
	$(MAKE) -C oracle clean

.PHONY: all oracle asm clean
