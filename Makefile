# Build: libskq.so (HIP kernels + C-ABI + C++ host), the skq CLI, and the test-only oracle.
ROCM    ?= /opt/rocm
HIPCC   ?= $(ROCM)/bin/hipcc
ARCH    ?= gfx950
PKG     := sketch-for-rna-seq_amd
CSRC    := $(PKG)/csrc
OUT     := $(PKG)/lib
CXXFLAGS_COMMON := -O3 -std=c++17 -fPIC -Wall -Iinclude -I$(CSRC)

oracle: oracle/liboracle.so
oracle/liboracle.so: oracle/oracle.c oracle/oracle.h
	gcc -O2 -Wall -Wextra -std=c11 -fPIC -shared -pthread $< -o $@

.PHONY: oracle

# the reference's own chain / EM / IO code, test-only (oracle/ref.mk; skipped without /root/reference),
# and the reference's own CLI (src/main.cpp) linked against libskq.so through include/dropin
ref: $(OUT)/libskq.so
	$(MAKE) -f oracle/ref.mk all
.PHONY: ref

HIPFLAGS := $(CXXFLAGS_COMMON) --offload-arch=$(ARCH) -munsafe-fp-atomics
LIB_OBJS := $(OUT)/obj/skq_kernels.o $(OUT)/obj/skq_map1.o $(OUT)/obj/skq_map1_pass.o $(OUT)/obj/skq_capi.o $(OUT)/obj/skq_tables.o $(OUT)/obj/skq_dropin.o \
            $(OUT)/obj/skq_io.o $(OUT)/obj/skq_ingest.o $(OUT)/obj/skq_em.o \
            $(OUT)/obj/skq_build.o $(OUT)/obj/skq_dropin_io.o $(OUT)/obj/skq_sketcher.o
HOST_CXX ?= g++
HOSTFLAGS := $(CXXFLAGS_COMMON) -pthread

lib: $(OUT)/libskq.so
$(OUT)/obj/%.o: $(CSRC)/%.hip $(CSRC)/skq_internal.h include/skq.h include/skq_host.h
	@mkdir -p $(OUT)/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
$(OUT)/obj/%.o: $(CSRC)/%.cpp $(CSRC)/skq_internal.h include/skq.h include/skq_host.h $(wildcard include/dropin/*.h)
	@mkdir -p $(OUT)/obj
	$(HOST_CXX) $(HOSTFLAGS) -c $< -o $@
# (the two map parts include skq_kernels.hip's helpers and skq_map1.h)
$(OUT)/obj/skq_map1.o $(OUT)/obj/skq_map1_pass.o: $(CSRC)/skq_kernels.hip $(CSRC)/skq_map1.h
$(OUT)/libskq.so: $(LIB_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -pthread -o $@ $(LIB_OBJS)

# development A/B builds (never the product): the kernel parts compiled with ABDEFS into
# $(OUT)/ab/$(AB)/libskq.so, loaded with SKQ_LIB; e.g. make ab AB=oldhash ABDEFS=-DSKQ_HASH_PAIR=0
AB ?= x
ABDEFS ?=
ABDIR := $(OUT)/ab/$(AB)
AB_KOBJS := $(ABDIR)/skq_kernels.o $(ABDIR)/skq_map1.o $(ABDIR)/skq_map1_pass.o
$(ABDIR)/%.o: $(CSRC)/%.hip $(CSRC)/skq_kernels.hip $(CSRC)/skq_map1.h $(CSRC)/skq_internal.h include/skq.h
	@mkdir -p $(ABDIR)
	$(HIPCC) $(HIPFLAGS) $(ABDEFS) -c $< -o $@
$(ABDIR)/libskq.so: $(AB_KOBJS) $(filter-out $(OUT)/obj/skq_kernels.o $(OUT)/obj/skq_map1.o $(OUT)/obj/skq_map1_pass.o,$(LIB_OBJS))
	$(HIPCC) --offload-arch=$(ARCH) -shared -pthread -o $@ $^
ab: $(ABDIR)/libskq.so
.PHONY: ab

# the debug build of the map's LDS slot counter (skq_map1.h lds_slot_next: clamped instead of
# wrapped below LDS address 0), loaded by tests/test_debug_lds_gpu.py through SKQ_LIB
DBG := $(OUT)/ab/debug_lds
$(DBG)/%.o: $(CSRC)/%.hip $(CSRC)/skq_kernels.hip $(CSRC)/skq_map1.h $(CSRC)/skq_internal.h include/skq.h
	@mkdir -p $(DBG)
	$(HIPCC) $(HIPFLAGS) -DSKQ_DEBUG_LDS=1 -c $< -o $@
$(DBG)/libskq.so: $(DBG)/skq_map1.o $(DBG)/skq_map1_pass.o $(filter-out $(OUT)/obj/skq_map1.o $(OUT)/obj/skq_map1_pass.o,$(LIB_OBJS))
	$(HIPCC) --offload-arch=$(ARCH) -shared -pthread -o $@ $^
debuglds: $(DBG)/libskq.so
.PHONY: debuglds

# the command line (index / quant), src/main.cpp's interface
# (several GPUs: HIP streams and RCCL from the host program; the HIP headers want the platform named)
$(OUT)/skq: $(CSRC)/skq_cli.cpp $(OUT)/libskq.so include/skq.h include/skq_host.h
	$(HOST_CXX) -O2 -std=c++17 -Wall -Iinclude -I$(ROCM)/include -D__HIP_PLATFORM_AMD__ $< -o $@ -L$(OUT) -lskq \
	    -L$(ROCM)/lib -lamdhip64 -lrccl -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(ROCM)/lib

# test driver for the C++ drop-in signatures (tests/test_dropin.py)
$(OUT)/skq_dropin_check: tests/dropin_check.cpp $(OUT)/libskq.so $(wildcard include/dropin/*.h)
	$(HOST_CXX) -O2 -std=c++17 -Wall -Iinclude/dropin $< -o $@ -L$(OUT) -lskq -Wl,-rpath,'$$ORIGIN'

all: lib oracle ref debuglds $(OUT)/skq $(OUT)/skq_dropin_check
.PHONY: lib all
.DEFAULT_GOAL := all
