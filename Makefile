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
	gcc -O2 -Wall -Wextra -std=c11 -fPIC -shared $< -o $@

.PHONY: oracle
