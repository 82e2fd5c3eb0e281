# Builds the product library kopia_amd/libkcdc.so (gfx950 only) and the C
# oracle used by the tests (oracle/_build/liboracle.so).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function
CSRC := kopia_amd/csrc
OBJ := build/obj
SRCS := $(CSRC)/kcdc_kernels.hip $(CSRC)/kcdc_hash.hip $(CSRC)/kcdc_crypt.hip $(CSRC)/kcdc_compress.hip $(CSRC)/kcdc_api.cpp $(CSRC)/kcdc_writer.cpp $(CSRC)/kcdc_tables.cpp $(CSRC)/kcdc_registry.cpp
OBJS := $(patsubst $(CSRC)/%,$(OBJ)/%.o,$(SRCS))
LIB := kopia_amd/libkcdc.so

all: $(LIB) oracle build/writer_bench

$(OBJ)/%.hip.o: $(CSRC)/%.hip $(CSRC)/kcdc_internal.h include/kcdc.h
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/%.cpp.o: $(CSRC)/%.cpp $(CSRC)/kcdc_internal.h include/kcdc.h
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJS)

oracle:
	$(MAKE) -s -C oracle

asm: $(CSRC)/kcdc_kernels.hip
	@mkdir -p build/asm
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S $< -o build/asm/kcdc_kernels.s -Rpass-analysis=kernel-resource-usage 2> build/asm/resource.txt

clean:
	rm -rf build $(LIB)
	$(MAKE) -s -C oracle clean

# Instrumented builds for tools/debug_pipe.py (queue invariants, KCDC_DEBUG_CHECKS) and
# tools/trace_pipe.py (per-wave s_memrealtime trace, KCDC_TRACE); not used by the product.
build/libkcdc_dbg.so build/libkcdc_trace.so: $(SRCS) $(CSRC)/kcdc_internal.h include/kcdc.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) $(if $(findstring dbg,$@),-DKCDC_DEBUG_CHECKS=1,-DKCDC_TRACE=1) -shared -o $@ \
	  $(CSRC)/kcdc_kernels.hip $(CSRC)/kcdc_hash.hip $(CSRC)/kcdc_crypt.hip $(CSRC)/kcdc_compress.hip \
	  -x hip $(CSRC)/kcdc_api.cpp $(CSRC)/kcdc_writer.cpp $(CSRC)/kcdc_tables.cpp $(CSRC)/kcdc_registry.cpp
instrumented: build/libkcdc_dbg.so build/libkcdc_trace.so
.PHONY: instrumented

# C ABI driver: concurrent writers through grouped vs private streaming handles
build/group_bench: tools/group_bench.cpp include/kcdc.h $(LIB)
	@mkdir -p build
	g++ -O2 -std=c++17 -pthread -Iinclude $< -Lkopia_amd -lkcdc -Wl,-rpath,'$$ORIGIN/../kopia_amd' -o $@

.PHONY: all oracle clean asm

# ---- experiment builds (A/B of compile-time tunables through tools/kbench.py; not the product)
# e.g. make variants VARIANTS="gap1:-DKCDC_HELP_GAP=1u lane1k:-DKCDC_LANE_MAX=1024"
VARIANTS ?=
variants:
	@mkdir -p build/variants
	@for v in $(VARIANTS); do \
	  n=$${v%%:*}; f=$$(echo $${v#*:} | tr ',' ' '); \
	  echo "variant $$n: $$f"; \
	  $(HIPCC) $(HIPFLAGS) $$f -shared -o build/variants/libkcdc_$$n.so $(CSRC)/kcdc_kernels.hip $(CSRC)/kcdc_hash.hip $(CSRC)/kcdc_crypt.hip $(CSRC)/kcdc_compress.hip -x hip $(CSRC)/kcdc_api.cpp $(CSRC)/kcdc_writer.cpp $(CSRC)/kcdc_tables.cpp $(CSRC)/kcdc_registry.cpp || exit 1; \
	done
.PHONY: variants

# C ABI driver: batching object writers (kcdc_bw_*), aggregate host-to-cuts rate
build/writer_bench: tools/writer_bench.cpp include/kcdc.h $(LIB)
	@mkdir -p build
	g++ -O2 -std=c++17 -pthread -Iinclude $< -Lkopia_amd -lkcdc -Wl,-rpath,'$$ORIGIN/../kopia_amd' -o $@

# Microbenchmarks run by tools/gpu_session.sh (valu:, membench): standalone HIP programs
build/valu_rate: tools/valu_rate.hip
	@mkdir -p build
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) $< -o $@
build/membench: tools/membench.hip
	@mkdir -p build
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) $< -o $@
tools: build/valu_rate build/membench build/writer_bench
.PHONY: tools
