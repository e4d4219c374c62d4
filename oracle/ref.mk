# Test-only builds of the reference's own code (NOT the product, never linked by it), compiled
# unmodified where the sources lie, outputs only into oracle/_ref/ (git-ignored):
#  * libref.so: src/{sparse_chaining,data_io,isoform_assignment}.cpp + oracle/ref_harness.cpp (a
#    C-ABI shim for ctypes) — the chain / EM / IO legs of the oracle's pinning;
#  * ref_cli_skq: the drop-in check of INTEGRATION.md §2 — the reference's CLI src/main.cpp with its
#    own data_io.cpp and isoform_assignment.cpp, kmer/sketch/sparse_chaining (and libnthash)
#    replaced by libskq.so through include/dropin (include/dropin/nthash/nthash.hpp stands for
#    <nthash/nthash.hpp>, which main.cpp includes);
#  * ref_cli_skq_all: src/main.cpp alone over libskq.so (data_io and isoform_assignment too).
# -include chrono/algorithm: src/main.cpp uses std::chrono and std::max_element without including
# their headers (it builds on libc++, which pulls them in transitively; libstdc++ does not).
# kmer.cpp / sketch.cpp need the absent ntHash library and are never built.
# usage: make -f oracle/ref.mk all   (a no-op when /root/reference is absent, e.g. on the GPU box)
REF     ?= /root/reference
OUTDIR  := oracle/_ref
LIBDIR  := sketch-for-rna-seq_amd/lib
REF_SRC := $(REF)/src/sparse_chaining.cpp $(REF)/src/data_io.cpp $(REF)/src/isoform_assignment.cpp
CLI_FLAGS := -std=c++17 -O2 -include chrono -include algorithm -Iinclude/dropin -I$(REF)/include
CLI_LINK  := -L$(LIBDIR) -lskq -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'
DROPIN_H  := $(wildcard include/dropin/*.h include/dropin/nthash/*.hpp)

ifneq ($(wildcard $(REF)/src/sparse_chaining.cpp),)
$(OUTDIR)/libref.so: oracle/ref_harness.cpp $(REF_SRC)
	@mkdir -p $(OUTDIR)
	g++ -std=c++17 -O2 -fPIC -shared -I$(REF)/include oracle/ref_harness.cpp $(REF_SRC) -o $@
$(OUTDIR)/ref_cli_skq: $(REF)/src/main.cpp $(REF)/src/data_io.cpp $(REF)/src/isoform_assignment.cpp $(LIBDIR)/libskq.so $(DROPIN_H)
	@mkdir -p $(OUTDIR)
	g++ $(CLI_FLAGS) $(REF)/src/main.cpp $(REF)/src/data_io.cpp $(REF)/src/isoform_assignment.cpp -o $@ $(CLI_LINK)
$(OUTDIR)/ref_cli_skq_all: $(REF)/src/main.cpp $(LIBDIR)/libskq.so $(DROPIN_H)
	@mkdir -p $(OUTDIR)
	g++ $(CLI_FLAGS) $(REF)/src/main.cpp -o $@ $(CLI_LINK)
all: $(OUTDIR)/libref.so $(OUTDIR)/ref_cli_skq $(OUTDIR)/ref_cli_skq_all
else
all:
	@echo "reference sources absent: oracle/_ref not built"
endif
.PHONY: all
.DEFAULT_GOAL := all
