# Builds the product library (gfx950 HIP) and the CPU oracle (test
# infrastructure).  `python -c "import __graft_entry__ as g; g.build()"` runs this.
HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
PKG     := noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd
ARCH    ?= gfx950
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -shared -std=c++17 -Wall -Wno-unused-result
HIPCFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Wall -Wno-unused-result
# `make DEV=1 ...`: development A/B build whose dtc_open honours the layout /
# geometry override variables (DTC_OCTET_BITS, DTC_LC_SPLIT, DTC_LC_TPB,
# DTC_KDK_SPLIT, DTC_BATCH_BYTES, DTC_NO_BASIS_SYNTH); never the product
ifeq ($(DEV),1)
HIPCFLAGS += -DDTC_DEV_KNOBS $(DEVFLAGS)
endif
# `make KNOMERGE=1`: kernel translation units without SI load/store merging
# (development A/B: with additive LDS slots, -DDTC_ADD_SLOTS, the re-layouts'
# accesses then keep their immediate offsets instead of pairing into
# ds_read2_b64; r4d: C2 -1.9 % against the product's XOR slots, merged).  The
# host pass of these units reports the feature as unknown and ignores it.
ifeq ($(KNOMERGE),1)
KFLAGS := -Xclang -target-feature -Xclang -load-store-opt
endif
# CPU oracle (test infrastructure): portable build, plus an x86-64-v3 build
# that is loaded only on hosts with those features.
ORACLE_MARCH ?= x86-64-v2
OBJDIR  := build/obj

LIB     := $(PKG)/lib/libdtc_hip.so
ORACLE  := oracle/liboracle.so
ORACLE3 := oracle/liboracle_v3.so
SRCS    := $(PKG)/csrc/dtc_kernels.hip $(PKG)/csrc/dtc_lightcone.hip $(PKG)/csrc/dtc_tile13.hip $(PKG)/csrc/dtc_engine.cpp
HDRS    := $(PKG)/csrc/dtc_kernels.h $(PKG)/csrc/dtc_device.h $(PKG)/csrc/dtc_rng.h include/dtc.h

all: $(LIB) $(ORACLE) $(ORACLE3)

# the two translation units compile separately (the kernels take minutes, the
# host engine seconds), then link into the one product library
$(OBJDIR)/dtc_kernels.o: $(PKG)/csrc/dtc_kernels.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	@rm -f $@
	$(HIPCC) $(HIPCFLAGS) $(KFLAGS) -c $< -o $@ 2> $@.log; rc=$$?; grep -v "not a recognized feature" $@.log >&2; exit $$rc

$(OBJDIR)/dtc_lightcone.o: $(PKG)/csrc/dtc_lightcone.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	@rm -f $@
	$(HIPCC) $(HIPCFLAGS) $(KFLAGS) -c $< -o $@ 2> $@.log; rc=$$?; grep -v "not a recognized feature" $@.log >&2; exit $$rc

$(OBJDIR)/dtc_tile13.o: $(PKG)/csrc/dtc_tile13.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	@rm -f $@
	$(HIPCC) $(HIPCFLAGS) $(KFLAGS) -c $< -o $@ 2> $@.log; rc=$$?; grep -v "not a recognized feature" $@.log >&2; exit $$rc

$(OBJDIR)/dtc_engine.o: $(PKG)/csrc/dtc_engine.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPCFLAGS) -c $< -o $@

$(LIB): $(OBJDIR)/dtc_kernels.o $(OBJDIR)/dtc_lightcone.o $(OBJDIR)/dtc_tile13.o $(OBJDIR)/dtc_engine.o
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared $^ -o $@

$(ORACLE): oracle/dtc_oracle.c
	$(CC) -O3 -march=$(ORACLE_MARCH) -fopenmp -fPIC -shared -std=c11 -Wall $< -o $@ -lm

# the same source for AVX2/FMA hosts: oracle/c_oracle.py loads it only when
# /proc/cpuinfo lists the x86-64-v3 features (the bench's CPU baseline)
$(ORACLE3): oracle/dtc_oracle.c
	$(CC) -O3 -march=x86-64-v3 -fopenmp -fPIC -shared -std=c11 -Wall $< -o $@ -lm

resource-usage: $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -Rpass-analysis=kernel-resource-usage $(SRCS) -o /tmp/dtc_ru.so

# Development-only build (instrumentation; never the product): per-workgroup
# phase timing, loaded with DTC_LIB=build/libdtc_timing.so by tools/phase_timing.py.
build/libdtc_timing.so: $(SRCS) $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -DDTC_PHASE_TIMING=3 $(SRCS) -o $@

clean:
	rm -f $(LIB) $(ORACLE) $(ORACLE3) $(OBJDIR)/*.o

.PHONY: all clean resource-usage
