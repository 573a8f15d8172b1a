# Builds the product library (gfx950 HIP) and the CPU oracle (test
# infrastructure).  `python -c "import __graft_entry__ as g; g.build()"` runs this.
HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
PKG     := noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd
ARCH    ?= gfx950
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -shared -std=c++17 -Wall -Wno-unused-result

LIB     := $(PKG)/lib/libdtc_hip.so
ORACLE  := oracle/liboracle.so
SRCS    := $(PKG)/csrc/dtc_kernels.hip $(PKG)/csrc/dtc_engine.cpp
HDRS    := $(PKG)/csrc/dtc_kernels.h $(PKG)/csrc/dtc_rng.h include/dtc.h

all: $(LIB) $(ORACLE)

$(LIB): $(SRCS) $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(SRCS) -o $@

$(ORACLE): oracle/dtc_oracle.c
	$(CC) -O3 -march=x86-64-v3 -fopenmp -fPIC -shared -std=c11 -Wall $< -o $@ -lm

resource-usage: $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -Rpass-analysis=kernel-resource-usage $(SRCS) -o /tmp/dtc_ru.so

# Development-only build (instrumentation; never the product): per-workgroup
# phase timing, loaded with DTC_LIB=build/libdtc_timing.so by tools/phase_timing.py.
build/libdtc_timing.so: $(SRCS) $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -DDTC_PHASE_TIMING=3 $(SRCS) -o $@

clean:
	rm -f $(LIB) $(ORACLE)

.PHONY: all clean resource-usage
