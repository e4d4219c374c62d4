# Test-only build of the reference's own code (NOT the product, never linked by it):
# /root/reference/src/{sparse_chaining,data_io,isoform_assignment}.cpp compiled unmodified where
# they lie, plus oracle/ref_harness.cpp (a C-ABI shim for ctypes), into oracle/_ref/libref.so.
# kmer.cpp / sketch.cpp / main.cpp need the absent ntHash library and are not built.
# usage: make -f oracle/ref.mk   (a no-op when /root/reference is absent, e.g. on the GPU box)
REF     ?= /root/reference
OUTDIR  := oracle/_ref
REF_SRC := $(REF)/src/sparse_chaining.cpp $(REF)/src/data_io.cpp $(REF)/src/isoform_assignment.cpp

ifneq ($(wildcard $(REF)/src/sparse_chaining.cpp),)
$(OUTDIR)/libref.so: oracle/ref_harness.cpp $(REF_SRC)
	@mkdir -p $(OUTDIR)
	g++ -std=c++17 -O2 -fPIC -shared -I$(REF)/include oracle/ref_harness.cpp $(REF_SRC) -o $@
else
$(OUTDIR)/libref.so:
	@echo "reference sources absent: oracle/_ref not built"
endif
.PHONY: all
all: $(OUTDIR)/libref.so
.DEFAULT_GOAL := $(OUTDIR)/libref.so
