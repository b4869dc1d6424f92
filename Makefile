# Top-level build: the gfx950 product library and the CPU oracle (test infra).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-inline-asm -fvisibility=hidden --offload-arch=$(ARCH) -Iinclude
LIBDIR := xsknf_amd/lib
LIB := $(LIBDIR)/libxsknf_gpu.so
SRCS := xsknf_amd/csrc/checksummer.hip xsknf_amd/csrc/host_path.hip xsknf_amd/csrc/multi.hip xsknf_amd/csrc/shard_plan.cpp
# RCCL for the multi-device calls (xsknf_gpu_multi_*)
GPULIBS := -L/opt/rocm/lib -lrccl

# host side: the AF_XDP runtime (plain C) and the checksummer NF binary
CC ?= gcc
CFLAGS ?= -O2 -g -std=gnu11 -Wall -Wextra -fPIC -fvisibility=hidden -Iinclude
RTLIB := $(LIBDIR)/libxsknf.so
RTSRCS := xsknf_amd/csrc/xsknf_rt.c xsknf_amd/csrc/rt_netlink.c
RTHDRS := include/xsknf.h xsknf_amd/csrc/xsk_ring.h xsknf_amd/csrc/rt_netlink.h
APP := xsknf_amd/bin/checksummer

all: $(LIB) $(RTLIB) $(APP) oracle

ASM := build/asm/checksummer-gfx950.s

# The library is kept only if the device code passes tools/check_inflight.py:
# no instruction may name a register of an inline-asm load before its counted
# s_waitcnt (the compiler does not know those registers are still in flight).
$(LIB): $(SRCS) include/xsknf_gpu.h xsknf_amd/csrc/checksummer_internal.h xsknf_amd/csrc/checksummer_ab.h tools/check_inflight.py Makefile
	@mkdir -p $(LIBDIR) build/asm
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S -o $(ASM) xsknf_amd/csrc/checksummer.hip
	python3 tools/check_inflight.py $(ASM)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(SRCS) $(GPULIBS)

$(RTLIB): $(RTSRCS) $(RTHDRS) Makefile
	@mkdir -p $(LIBDIR)
	$(CC) $(CFLAGS) -shared -pthread -o $@ $(RTSRCS)

$(APP): xsknf_amd/csrc/checksummer_app.c $(RTLIB) $(LIB) include/xsknf.h include/xsknf_gpu.h
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -o $@ $< -L$(LIBDIR) -lxsknf -lxsknf_gpu -Wl,-rpath,'$$ORIGIN/../lib' -pthread

# config-1 harness (test / measurement infra: links the CPU oracle as the NF)
VETH := tools/build/xsk_veth
PROBE := tools/build/hbm_probe
PROBELIB := tools/build/libhbm_probe.so
HOOKBENCH := tools/build/hook_bench
CTXLAT := tools/build/ctx_latency
BARPROBE := tools/build/bar_probe
DEVPROBE := tools/build/dev_probe
MULTIC4 := tools/build/multi_config4
tools: $(VETH) $(PROBE) $(PROBELIB) $(HOOKBENCH) $(CTXLAT) $(BARPROBE) $(DEVPROBE) $(MULTIC4)
# config 4 through the multi-device calls from a C host (checked against the CPU oracle)
$(MULTIC4): tools/multi_config4.c $(LIB) oracle
	@mkdir -p $(dir $@)
	$(CC) -O2 -g -std=gnu11 -Wall -Wextra -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ $< \
		-L$(LIBDIR) -lxsknf_gpu -Loracle/build -lcsum_oracle -L/opt/rocm/lib -lamdhip64 \
		-Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,'$$ORIGIN/../../oracle/build' -Wl,-rpath,/opt/rocm/lib
# one NF-shaped process start (device count, a context), for tools/nf_start_probe.py
$(DEVPROBE): tools/dev_probe.c $(LIB)
	@mkdir -p $(dir $@)
	$(CC) -O2 -g -std=gnu11 -Wall -Wextra -Iinclude -o $@ $< -L$(LIBDIR) -lxsknf_gpu \
		-Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'
$(BARPROBE): tools/bar_probe.hip
	@mkdir -p $(dir $@)
	$(HIPCC) -O2 -std=c++17 --offload-arch=$(ARCH) -o $@ $<
$(PROBE): tools/hbm_probe.hip
	@mkdir -p $(dir $@)
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -Wno-inline-asm -o $@ $<
$(PROBELIB): tools/hbm_probe.hip
	@mkdir -p $(dir $@)
	$(HIPCC) -O3 -std=c++17 -fPIC -shared -fvisibility=hidden -DHBM_PROBE_LIB --offload-arch=$(ARCH) -Wno-inline-asm -o $@ $<
$(VETH): tools/xsk_veth.c xsknf_amd/csrc/rt_netlink.c $(RTLIB) oracle
	@mkdir -p $(dir $@)
	$(CC) -O2 -g -std=gnu11 -Wall -Wextra -Iinclude -o $@ tools/xsk_veth.c xsknf_amd/csrc/rt_netlink.c \
		-L$(LIBDIR) -lxsknf -Loracle/build -lcsum_oracle \
		-Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,'$$ORIGIN/../../oracle/build' -pthread -ldl

# NF-level rate of the worker loop with the GPU hook (one-call / two-phase) or the CPU NF
$(HOOKBENCH): tools/hook_bench.c $(RTLIB) $(LIB) oracle
	@mkdir -p $(dir $@)
	$(CC) -O2 -g -std=gnu11 -Wall -Wextra -Iinclude -o $@ tools/hook_bench.c \
		-L$(LIBDIR) -lxsknf -lxsknf_gpu -Loracle/build -lcsum_oracle \
		-Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,'$$ORIGIN/../../oracle/build' -pthread -ldl

$(CTXLAT): tools/ctx_latency.c $(LIB)
	@mkdir -p $(dir $@)
	$(CC) -O2 -g -std=gnu11 -Wall -Wextra -Iinclude -o $@ $< -L$(LIBDIR) -lxsknf_gpu -pthread \
		-Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

# A/B build: every kernel family and launch shape (tools/tune.py, tools/ab_libs.sh;
# XSKNF_GPU_LIB=build/ab/libxsknf_gpu.so selects it).  Not the product.
ABLIB := build/ab/libxsknf_gpu.so
ab: $(ABLIB)
$(ABLIB): $(SRCS) include/xsknf_gpu.h xsknf_amd/csrc/checksummer_internal.h xsknf_amd/csrc/checksummer_ab.h tools/check_inflight.py Makefile
	@mkdir -p build/ab
	$(HIPCC) $(HIPFLAGS) -DXSKNF_AB --cuda-device-only -S -o build/ab/checksummer-gfx950.s xsknf_amd/csrc/checksummer.hip
	python3 tools/check_inflight.py build/ab/checksummer-gfx950.s
	$(HIPCC) $(HIPFLAGS) -DXSKNF_AB -shared -o $@ $(SRCS) $(GPULIBS)

# Timeline build: the product shapes with the split kernel's per-wave clock
# samples (tools/timeline.py).  Not the product.
TLLIB := build/tl/libxsknf_gpu.so
tl: $(TLLIB)
$(TLLIB): $(SRCS) include/xsknf_gpu.h xsknf_amd/csrc/checksummer_internal.h xsknf_amd/csrc/checksummer_ab.h tools/check_inflight.py Makefile
	@mkdir -p build/tl
	$(HIPCC) $(HIPFLAGS) -DXSKNF_TIMELINE $(TLFLAGS) --cuda-device-only -S -o build/tl/checksummer-gfx950.s xsknf_amd/csrc/checksummer.hip
	python3 tools/check_inflight.py build/tl/checksummer-gfx950.s
	$(HIPCC) $(HIPFLAGS) -DXSKNF_TIMELINE $(TLFLAGS) -shared -o $@ $(SRCS) $(GPULIBS)

# keep the device assembly for inspection (VGPRs, instruction mix)
asm: $(SRCS)
	@mkdir -p build/asm
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S -o $(ASM) xsknf_amd/csrc/checksummer.hip

# the restatement, and (where the reference checkout exists) the reference's
# own per-packet function compiled from its verbatim lines (oracle/_ref)
REF ?= /root/reference
oracle:
	$(MAKE) -C oracle
	if [ -d $(REF)/examples/checksummer ]; then $(MAKE) -C oracle ref REF=$(REF); fi

clean:
	rm -rf $(LIBDIR) xsknf_amd/bin build
	$(MAKE) -C oracle clean

.PHONY: all oracle asm clean tools ab tl guard

# Guard build: every UMEM access of the split kernel's paths range-checked and
# recorded instead of faulting (tools/guard_run.py).  Not the product.
GDLIB := build/guard/libxsknf_gpu.so
guard: $(GDLIB)
$(GDLIB): $(SRCS) include/xsknf_gpu.h xsknf_amd/csrc/checksummer_internal.h Makefile
	@mkdir -p build/guard
	$(HIPCC) $(HIPFLAGS) -DXSKNF_GUARD -shared -o $@ $(SRCS) $(GPULIBS)
