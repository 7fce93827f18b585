# vcfx_amd build: HIP engine (libvcfx_gpu.so, gfx950), host core + tool binaries, synthetic
# generator.  Outputs under build/ (git-ignored, shipped to the GPU box by gpurun).
# The oracle (test infrastructure) has its own makefiles under oracle/.
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
CC ?= gcc
ARCH ?= gfx950
B := build
GPU_SRC := vcfx_amd/csrc/gpu
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Iinclude -I$(GPU_SRC) $(EXTRA_HIPFLAGS)
GPU_OBJS := $(B)/obj/vcfxg_kernels.o $(B)/obj/vcfxg_rf.o $(B)/obj/vcfxg_ld.o $(B)/obj/vcfxg_ld_fast.o $(B)/obj/vcfxg_ld_mask.o $(B)/obj/vcfxg_af_walk.o $(B)/obj/vcfxg_fq_walk.o $(B)/obj/vcfxg_hwe.o $(B)/obj/vcfxg_dose.o $(B)/obj/vcfxg_md.o $(B)/obj/vcfxg_ac.o $(B)/obj/vcfxg_ph.o $(B)/obj/vcfxg_inflate.o $(B)/obj/vcfxg_api.o $(B)/obj/vcfxg_decimal.o

TOOLS := VCFX_allele_freq_calc VCFX_genotype_query VCFX_record_filter VCFX_variant_counter VCFX_ld_calculator \
         VCFX_nonref_filter VCFX_hwe_tester VCFX_dosage_calculator VCFX_missing_detector VCFX_allele_counter \
         VCFX_haplotype_phaser
HOST_SRC := vcfx_amd/csrc/host
TOOL_SRC := vcfx_amd/csrc/tools
CXXFLAGS := -O2 -std=c++17 -fPIC -Wall -Wno-unused-result -Iinclude -I$(HOST_SRC) -I$(TOOL_SRC)
TOOL_OBJS := $(sort $(B)/obj/hostio.o $(B)/obj/gz.o $(patsubst $(TOOL_SRC)/%.cpp,$(B)/obj/%.o,$(wildcard $(TOOL_SRC)/tool_*.cpp)))
TOOL_BINS := $(foreach t,$(TOOLS),$(B)/src/$(t)/$(t))

all: $(B)/bin/vcfx_bgzf $(B)/bin/vcfx_drain $(B)/bin/vcfx_pipe_ceiling $(B)/bin/vcfx_pipe $(B)/libvcfx_gpu.so $(B)/libvcfx_tools.so $(TOOL_BINS) $(B)/bin/vcfx_synth $(B)/libvcfx_synth.so \
     $(B)/libvcfx_core.so $(B)/libvcfx_core.a $(B)/libvcfx_record_filter.so $(B)/libvcfx_genotype_query.so

$(B)/obj/%.o: $(HOST_SRC)/%.cpp $(wildcard $(HOST_SRC)/*.h) include/vcfx_gpu.h
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c -o $@ $<

$(B)/obj/%.o: $(TOOL_SRC)/%.cpp $(wildcard $(TOOL_SRC)/*.h) $(wildcard $(HOST_SRC)/*.h) include/vcfx_gpu.h
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c -o $@ $<

# libvcfx_core: the host vcfx:: core API (include/vcfx_core.h, include/vcfx_io.h)
$(B)/obj/core/vcfx_core.o: $(HOST_SRC)/vcfx_core.cpp include/vcfx_core.h include/vcfx_io.h
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -DVCFX_VERSION='"1.1.4"' -c -o $@ $<
$(B)/libvcfx_core.so: $(B)/obj/core/vcfx_core.o
	$(CXX) -shared -o $@ $< -lz
$(B)/libvcfx_core.a: $(B)/obj/core/vcfx_core.o
	ar rcs $@ $<

$(B)/libvcfx_tools.so: $(TOOL_OBJS) $(B)/libvcfx_gpu.so
	$(CXX) -shared -o $@ $(TOOL_OBJS) -L$(B) -lvcfx_gpu -lz -Wl,-rpath,'$$ORIGIN'

# the reference's per-tool library interfaces (include/vcfx_record_filter.h,
# include/vcfx_genotype_query.h): one library each, as each declares its own printHelp()
API_SRC := vcfx_amd/csrc/api
$(B)/obj/api_%.o: $(API_SRC)/%_api.cpp include/vcfx_%.h $(wildcard $(TOOL_SRC)/*.h) $(wildcard $(HOST_SRC)/*.h)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c -o $@ $<
$(B)/libvcfx_%.so: $(B)/obj/api_%.o $(B)/libvcfx_tools.so
	$(CXX) -shared -o $@ $< -L$(B) -lvcfx_tools -lvcfx_gpu -Wl,-rpath,'$$ORIGIN'

# drop-in executables at build/src/VCFX_<t>/VCFX_<t> (the reference test scripts' layout)
$(B)/src/%: $(TOOL_SRC)/binary_main.cpp $(B)/libvcfx_tools.so
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -DVCFX_TOOL_NAME='"$(notdir $@)"' -o $@ $< -L$(B) -lvcfx_tools -lvcfx_gpu -Wl,-rpath,'$$ORIGIN/../..'

$(B)/bin/vcfx_pipe: $(TOOL_SRC)/pipe_main.cpp $(B)/libvcfx_tools.so
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -o $@ $< -L$(B) -lvcfx_tools -lvcfx_gpu -Wl,-rpath,'$$ORIGIN/..'

$(B)/obj/vcfxg_%.o: $(GPU_SRC)/vcfxg_%.hip $(wildcard $(GPU_SRC)/*.h) include/vcfx_gpu.h
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(B)/obj/vcfxg_decimal.o: $(GPU_SRC)/vcfxg_decimal.cpp $(GPU_SRC)/vcfxg_decimal.h
	@mkdir -p $(dir $@)
	$(CXX) -O2 -std=c++17 -fPIC -Wall -c -o $@ $<

$(B)/libvcfx_gpu.so: $(GPU_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

$(B)/bin/vcfx_synth: vcfx_amd/csrc/synth/vcfx_synth.c
	@mkdir -p $(dir $@)
	$(CC) -O2 -DVCFX_SYNTH_MAIN -o $@ $< -lpthread

$(B)/bin/vcfx_bgzf: vcfx_amd/csrc/synth/vcfx_bgzf.c
	@mkdir -p $(dir $@)
	$(CC) -O2 -o $@ $< -lz -lpthread

$(B)/bin/vcfx_drain: tools/microbench/pipe_drain.c
	@mkdir -p $(dir $@)
	$(CC) -O2 -o $@ $<

# the drop-in's stdin reader with the device stage stubbed (the e2e leg's pipe ceiling)
PIPE_CEIL_SRC := tools/microbench/pipe_ceiling.cpp tests/shard_tsan_stub.cpp $(HOST_SRC)/hostio.cpp $(HOST_SRC)/gz.cpp
$(B)/bin/vcfx_pipe_ceiling: $(PIPE_CEIL_SRC) $(wildcard $(HOST_SRC)/*.h)
	@mkdir -p $(dir $@)
	$(CXX) -O2 -std=c++17 -DVCFX_STUB_DISCARD -Iinclude -I$(HOST_SRC) -Ivcfx_amd/csrc/tools -o $@ $(PIPE_CEIL_SRC) -lz -lpthread

$(B)/libvcfx_synth.so: vcfx_amd/csrc/synth/vcfx_synth.c
	$(CC) -O2 -fPIC -shared -o $@ $< -lpthread

clean:
	rm -rf $(B)
.PHONY: all clean

# host sanitizer builds (SURVEY §5 race detection): the input layer (hostio.cpp, gz.cpp:
# page-population, BGZF inflate, pipe reader threads) under ASan+UBSan and under TSan, and the
# vcfx:: core API under ASan+UBSan; run by tests/test_sanitize.py.  Host code only -- no GPU
# sanitizer on this pool.
SAN := $(B)/san
SANFLAGS := -O1 -g -fno-omit-frame-pointer -std=c++17 -Iinclude -I$(HOST_SRC)
SAN_HOST_SRC := tests/host_san_test.cpp $(HOST_SRC)/hostio.cpp $(HOST_SRC)/gz.cpp
sanitize: $(SAN)/host_san_asan $(SAN)/host_san_tsan $(SAN)/core_api_asan $(SAN)/shard_tsan $(SAN)/shard_asan
$(SAN)/host_san_asan: $(SAN_HOST_SRC) $(wildcard $(HOST_SRC)/*.h) $(B)/libvcfx_gpu.so
	@mkdir -p $(dir $@)
	$(CXX) $(SANFLAGS) -fsanitize=address,undefined -fno-sanitize-recover=undefined -o $@ $(SAN_HOST_SRC) \
	    -L$(B) -lvcfx_gpu -lz -lpthread -Wl,-rpath,'$$ORIGIN/..'
$(SAN)/host_san_tsan: $(SAN_HOST_SRC) $(wildcard $(HOST_SRC)/*.h) $(B)/libvcfx_gpu.so
	@mkdir -p $(dir $@)
	$(CXX) $(SANFLAGS) -fsanitize=thread -o $@ $(SAN_HOST_SRC) -L$(B) -lvcfx_gpu -lz -lpthread -Wl,-rpath,'$$ORIGIN/..'
$(SAN)/core_api_asan: tests/core_api_test.cpp $(HOST_SRC)/vcfx_core.cpp include/vcfx_core.h include/vcfx_io.h
	@mkdir -p $(dir $@)
	$(CXX) $(SANFLAGS) -fsanitize=address,undefined -fno-sanitize-recover=undefined \
	    -o $@ tests/core_api_test.cpp $(HOST_SRC)/vcfx_core.cpp -lz
# the in-process multi-GPU runner's host side (rank threads, getopt lock, thread-local ShardRank,
# the ordered output writer, the clique) with vcfxg_* replaced by a host stand-in
SHARD_SAN_SRC := tests/shard_tsan_stub.cpp vcfx_amd/csrc/tools/tool_shard_main.cpp \
    vcfx_amd/csrc/tools/tool_allele_freq_calc.cpp $(HOST_SRC)/hostio.cpp $(HOST_SRC)/gz.cpp
$(SAN)/shard_tsan: $(SHARD_SAN_SRC) $(wildcard $(HOST_SRC)/*.h) vcfx_amd/csrc/tools/tools.h
	@mkdir -p $(dir $@)
	$(CXX) $(SANFLAGS) -Ivcfx_amd/csrc/tools -fsanitize=thread -o $@ $(SHARD_SAN_SRC) -lz -lpthread
$(SAN)/shard_asan: $(SHARD_SAN_SRC) $(wildcard $(HOST_SRC)/*.h) vcfx_amd/csrc/tools/tools.h
	@mkdir -p $(dir $@)
	$(CXX) $(SANFLAGS) -Ivcfx_amd/csrc/tools -fsanitize=address,undefined -fno-sanitize-recover=undefined \
	    -o $@ $(SHARD_SAN_SRC) -lz -lpthread
.PHONY: sanitize
