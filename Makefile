# gsdr-mi355x build: libgsdr.so (HIP, gfx950) and the CPU oracle (plain C, test infrastructure only).
HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
ARCH    ?= gfx950
BUILD   := build

HIPFLAGS := -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=$(ARCH) -fvisibility=hidden -fvisibility-inlines-hidden \
            -Wall -Wno-unused-function -Iinclude -Igsdr_amd/csrc -munsafe-fp-atomics
# Oracle: explicit fmaf where the spec says FMA, no implicit contraction.
OFLAGS  := -O2 -std=c11 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wextra -Ioracle -mfma

SRCS := $(wildcard gsdr_amd/csrc/*.hip)
HDRS := $(wildcard gsdr_amd/csrc/*.hpp) $(wildcard gsdr_amd/csrc/*.inc) $(wildcard include/gsdr/*.h)
OBJS := $(patsubst gsdr_amd/csrc/%.hip,$(BUILD)/%.o,$(SRCS))

all: gsdr_amd/libgsdr.so oracle/build/liboracle.so examples probes

$(BUILD)/%.o: gsdr_amd/csrc/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

gsdr_amd/libgsdr.so: $(OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -Wl,-rpath,/opt/rocm/lib $(OBJS) -o $@

# Tuning-probe build: the product objects with fir.hip (ablation variants >= 100 of gsdrxFirFCVariant) and iir.hip
# (the single-pass IIR, gsdrxIirFFSinglePass / CC) recompiled under GSDR_TUNING_PROBES. Loaded by tools/, by
# bench.py's staging-ceiling leg and by tests/test_gpu_iir_single_pass.py; never by the product path.
probes: $(BUILD)/probes/libgsdr_probes.so

PROBE_SRCS := fir iir
PROBE_OBJS := $(patsubst %,$(BUILD)/probes/%.o,$(PROBE_SRCS))

$(BUILD)/probes/%.o: gsdr_amd/csrc/%.hip $(HDRS)
	@mkdir -p $(BUILD)/probes
	$(HIPCC) $(HIPFLAGS) -DGSDR_TUNING_PROBES -c $< -o $@

$(BUILD)/probes/libgsdr_probes.so: $(filter-out $(patsubst %,$(BUILD)/%.o,$(PROBE_SRCS)),$(OBJS)) $(PROBE_OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -Wl,-rpath,/opt/rocm/lib $^ -o $@

oracle/build/liboracle.so: oracle/gsdr_oracle.c oracle/gsdr_oracle.h gsdr_amd/csrc/awgn_table.inc gsdr_amd/csrc/awgn_tail_table.inc
	@mkdir -p oracle/build
	$(CC) $(OFLAGS) -shared oracle/gsdr_oracle.c -o $@ -lm -lpthread

# C++ host example linking the C ABI
examples: $(BUILD)/fm_receiver $(BUILD)/short_call_timer

$(BUILD)/fm_receiver: examples/fm_receiver.cpp gsdr_amd/libgsdr.so $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) -O2 -std=c++17 -Iinclude $< -Lgsdr_amd -lgsdr -Wl,-rpath,'$$ORIGIN/../gsdr_amd' -o $@

$(BUILD)/short_call_timer: examples/short_call_timer.cpp gsdr_amd/libgsdr.so $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) -O2 -std=c++17 -Iinclude $< -Lgsdr_amd -lgsdr -Wl,-rpath,'$$ORIGIN/../gsdr_amd' -o $@

clean:
	rm -rf $(BUILD) gsdr_amd/libgsdr.so oracle/build

.PHONY: all clean examples probes
