# Builds libmchecksum.so (the drop-in mchecksum C ABI + MI355X batch kernels),
# libmchecksum_bench.so (device-side synthetic data for tests/bench) and the
# CPU oracle (test infrastructure, oracle/_build).  gfx950 only.
HIPCC     ?= /opt/rocm/bin/hipcc
CC        ?= gcc
ARCH      ?= gfx950
BUILD     := build
LIBDIR    := mercury_amd/lib
CSRC      := mercury_amd/csrc
INC       := -Iinclude -I$(CSRC)
CFLAGS    ?= -O2 -g -std=c11 -Wall -Wextra -fPIC -fvisibility=hidden
HIPFLAGS  ?= -O3 -g --offload-arch=$(ARCH) -fPIC -fvisibility=hidden -std=c++17 -Wall \
             -munsafe-fp-atomics
EXTRA_HIPFLAGS ?=

LIB       := $(LIBDIR)/libmchecksum.so
BENCHLIB  := $(LIBDIR)/libmchecksum_bench.so
COBJS     := $(BUILD)/mchecksum_cpu.o $(BUILD)/mchecksum_models.o $(BUILD)/crc_tables.o
GOBJS     := $(BUILD)/mchecksum_gpu.o $(BUILD)/mchecksum_gpu_ext.o

QFAULTLIB := $(BUILD)/libmchecksum_qfault.so

# Source digest compiled into the libraries (tools/src_digest.py): a test
# compares it with the tree, so the tested binary is provably HEAD's sources.
STAMP_SRCS := $(sort $(wildcard $(CSRC)/*.c $(CSRC)/*.h $(CSRC)/*.hip include/*.h))
STAMP     := $(BUILD)/src_stamp.o

all: $(LIB) $(BENCHLIB) oracle $(BUILD)/c1_bench $(QFAULTLIB) $(BUILD)/libcpu_batch.so $(BUILD)/hg_verify_consumer

$(BUILD) $(LIBDIR):
	mkdir -p $@

$(BUILD)/%.o: $(CSRC)/%.c $(wildcard $(CSRC)/*.h) include/mchecksum.h | $(BUILD)
	$(CC) $(CFLAGS) $(INC) -c $< -o $@

$(BUILD)/mchecksum_gpu.o: $(CSRC)/mchecksum_gpu.hip $(wildcard $(CSRC)/*.h) include/mchecksum_gpu.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(EXTRA_HIPFLAGS) $(INC) -c $< -o $@

$(BUILD)/mchecksum_gpu_ext.o: $(CSRC)/mchecksum_gpu_ext.hip $(wildcard $(CSRC)/*.h) include/mchecksum_gpu.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(EXTRA_HIPFLAGS) $(INC) -c $< -o $@

$(BUILD)/bench_datagen.o: $(CSRC)/bench_datagen.hip | $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(INC) -c $< -o $@

$(BUILD)/src_stamp.c: $(STAMP_SRCS) tools/src_digest.py | $(BUILD)
	python3 tools/src_digest.py --c-source $@ $(STAMP_SRCS)

$(STAMP): $(BUILD)/src_stamp.c
	$(CC) $(CFLAGS) -c $< -o $@

$(LIB): $(COBJS) $(GOBJS) $(STAMP) | $(LIBDIR)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -lpthread -Wl,-soname,libmchecksum.so.2
	ln -sf libmchecksum.so $(LIBDIR)/libmchecksum.so.2

# Test-only build: the work queue gives up one wait per launch
# (MCK_QFAULT_TEST, crc_gpu_device.h), loaded by tests/test_gpu_fail_closed.py
# next to the product library to check that such a launch fails closed.
$(BUILD)/qfault_gpu.o: $(CSRC)/mchecksum_gpu.hip $(wildcard $(CSRC)/*.h) include/mchecksum_gpu.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DMCK_QFAULT_TEST=1 $(INC) -c $< -o $@

$(BUILD)/qfault_gpu_ext.o: $(CSRC)/mchecksum_gpu_ext.hip $(wildcard $(CSRC)/*.h) include/mchecksum_gpu.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DMCK_QFAULT_TEST=1 $(INC) -c $< -o $@

$(QFAULTLIB): $(COBJS) $(BUILD)/qfault_gpu.o $(BUILD)/qfault_gpu_ext.o $(STAMP)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -lpthread

$(BENCHLIB): $(BUILD)/bench_datagen.o $(STAMP) | $(LIBDIR)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^

oracle:
	$(MAKE) -C oracle

$(BUILD)/c1_bench: tools/c1_bench.c include/mchecksum.h $(LIB) | $(BUILD)
	$(CC) -O2 -std=c11 -Wall -Iinclude $< -o $@ -L$(LIBDIR) -lmchecksum -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'

# bench.py's cpu_baseline "product" leg: the streaming API over a batch on n threads
$(BUILD)/libcpu_batch.so: tools/cpu_batch.c include/mchecksum.h $(LIB) | $(BUILD)
	$(CC) -O2 -std=c11 -Wall -Wextra -fPIC -shared -fvisibility=hidden -Iinclude $< -o $@ -L$(LIBDIR) -lmchecksum \
	  -lpthread -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'

# A compiled consumer of the batch ABI, found
# through cmake/mchecksum-config.cmake as Mercury would; run by
# tests/test_gpu_consumer.py on the GPU and tests/test_cmake_consumer.py here.
$(BUILD)/hg_verify_consumer: tests/native/hg_verify_consumer.c tests/native/hg_consumer/CMakeLists.txt \
		include/mchecksum.h include/mchecksum_gpu.h cmake/mchecksum-config.cmake $(LIB) | $(BUILD)
	cmake -S tests/native/hg_consumer -B $(BUILD)/hg_consumer -Dmchecksum_DIR=$(CURDIR)/cmake > /dev/null
	cmake --build $(BUILD)/hg_consumer > /dev/null
	cp $(BUILD)/hg_consumer/hg_verify_consumer $@

# CPU-only artefacts (no hipcc needed): streaming API for host tests.
cpu: $(LIBDIR)/libmchecksum_cpu.so
$(LIBDIR)/libmchecksum_cpu.so: $(COBJS) | $(LIBDIR)
	$(CC) -shared -o $@ $^ -lpthread

# Disassembly for roofline/occupancy inspection.
asm: | $(BUILD)
	cd $(BUILD) && $(HIPCC) $(HIPFLAGS) $(EXTRA_HIPFLAGS) -I../include -I../$(CSRC) --save-temps \
	  -c ../$(CSRC)/mchecksum_gpu.hip -o asm_tmp.o \
	  -Rpass-analysis=kernel-resource-usage 2> resource_usage.txt; \
	rm -f mchecksum_gpu-host-* mchecksum_gpu.hip-hip-*; true

clean:
	rm -rf $(BUILD) $(LIBDIR)/*.so
	$(MAKE) -C oracle clean

.PHONY: all oracle clean cpu asm

# A/B variants of the batch kernels (tools/ab_variants.py).  Each is a full
# libmchecksum built with different tuning macros.
VARIANTS ?= base:
variants: $(COBJS) $(BUILD)/mchecksum_gpu_ext.o | $(BUILD)
	mkdir -p $(BUILD)/variants
	@for v in $(VARIANTS); do n=$${v%%:*}; f=$$(echo $${v#*:} | tr , " "); \
	  echo "variant $$n: $$f"; \
	  $(HIPCC) $(HIPFLAGS) $$f $(INC) -c $(CSRC)/mchecksum_gpu.hip -o $(BUILD)/variants/gpu_$$n.o && \
	  $(HIPCC) $(HIPFLAGS) $$f $(INC) -c $(CSRC)/mchecksum_gpu_ext.hip -o $(BUILD)/variants/gpu_ext_$$n.o && \
	  $(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $(BUILD)/variants/libmchecksum_$$n.so $(COBJS) $(BUILD)/variants/gpu_$$n.o $(BUILD)/variants/gpu_ext_$$n.o -lpthread || exit 1; \
	done
.PHONY: variants

# The committed kernel sources at $(PREV) (all of csrc/ and include/) as
# variant "prev" (A/B against the last commit).  Its C objects are rebuilt
# from the same sources: the table packs are shared structs.
PREV ?= HEAD
prev: $(COBJS) | $(BUILD)
	rm -rf $(BUILD)/variants/prev_src && mkdir -p $(BUILD)/variants/prev_src
	git archive $(PREV) mercury_amd/csrc include | tar -x -C $(BUILD)/variants/prev_src
	$(HIPCC) $(HIPFLAGS) -I$(BUILD)/variants/prev_src/include -I$(BUILD)/variants/prev_src/$(CSRC) \
	  -c $(BUILD)/variants/prev_src/$(CSRC)/mchecksum_gpu.hip -o $(BUILD)/variants/gpu_prev.o
	$(HIPCC) $(HIPFLAGS) -I$(BUILD)/variants/prev_src/include -I$(BUILD)/variants/prev_src/$(CSRC) \
	  -c $(BUILD)/variants/prev_src/$(CSRC)/mchecksum_gpu_ext.hip -o $(BUILD)/variants/gpu_ext_prev.o
	for f in $(notdir $(COBJS:.o=)); do $(CC) $(CFLAGS) -I$(BUILD)/variants/prev_src/include \
	  -I$(BUILD)/variants/prev_src/$(CSRC) -c $(BUILD)/variants/prev_src/$(CSRC)/$$f.c \
	  -o $(BUILD)/variants/prev_$$f.o || exit 1; done
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $(BUILD)/variants/libmchecksum_prev.so \
	  $(addprefix $(BUILD)/variants/prev_,$(notdir $(COBJS))) \
	  $(BUILD)/variants/gpu_prev.o $(BUILD)/variants/gpu_ext_prev.o -lpthread
	cp $(LIB) $(BUILD)/variants/libmchecksum_cur.so
.PHONY: variants prev
