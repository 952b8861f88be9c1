# Build of the MI355X topic-routing engine (gfx950 only) and its test oracle.
#   emqx_amd/libtopicmatch.so  product: C-ABI + HIP kernels (hipcc, gfx950)
#   emqx_amd/libtmwork.so      synthetic workload generator (bench/test input)
#   oracle/liboracle.so        CPU restatement of the reference (checker only)
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
CC      ?= gcc
TMDEFS  ?=
HIPFLAGS = --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Wall -Wno-unused-result $(TMDEFS)
BUILD   ?= build
LIBOUT  ?= emqx_amd/libtopicmatch.so

all: $(LIBOUT) emqx_amd/libtmwork.so oracle/liboracle.so tools/ubench/batcher_bench tools/ubench/libbatchdrive.so

$(BUILD):
	mkdir -p $(BUILD)

$(BUILD)/kernels.o: emqx_amd/csrc/kernels.hip emqx_amd/csrc/kernels.h emqx_amd/csrc/image.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/engine.o: emqx_amd/csrc/engine.cpp emqx_amd/csrc/kernels.h emqx_amd/csrc/image.h include/topicmatch.h | $(BUILD)
	$(HIPCC) -O3 -fPIC -std=c++17 -Wall $(TMDEFS) -c $< -o $@

# A/B builds of compile-time variants: make variant TAG=x TMDEFS="-D..." ->
# emqx_amd/variants/libtopicmatch_x.so (bench.py --lib)
variant:
	mkdir -p emqx_amd/variants
	$(MAKE) BUILD=build_$(TAG) LIBOUT=emqx_amd/variants/libtopicmatch_$(TAG).so TMDEFS="$(TMDEFS)" emqx_amd/variants/libtopicmatch_$(TAG).so
.PHONY: variant

$(BUILD)/shard.o: emqx_amd/csrc/shard.hip emqx_amd/csrc/kernels.h emqx_amd/csrc/image.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/routes.o: emqx_amd/csrc/routes.hip emqx_amd/csrc/kernels.h emqx_amd/csrc/image.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/presort.o: emqx_amd/csrc/presort.hip emqx_amd/csrc/kernels.h emqx_amd/csrc/image.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/aggre.o: emqx_amd/csrc/aggre.hip emqx_amd/csrc/kernels.h emqx_amd/csrc/image.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/exchange.o: emqx_amd/csrc/exchange.cpp emqx_amd/csrc/kernels.h include/topicmatch.h | $(BUILD)
	$(HIPCC) -O2 -fPIC -std=c++17 -Wall -c $< -o $@

$(BUILD)/batcher.o: emqx_amd/csrc/batcher.cpp include/topicmatch.h | $(BUILD)
	$(HIPCC) -O2 -fPIC -std=c++17 -Wall -pthread -c $< -o $@

$(BUILD)/route.o: emqx_amd/csrc/route.hip emqx_amd/csrc/kernels.h emqx_amd/csrc/image.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/acl.o: emqx_amd/csrc/acl.hip include/topicmatch.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/rewrite.o: emqx_amd/csrc/rewrite.hip include/topicmatch.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBOUT): $(BUILD)/kernels.o $(BUILD)/shard.o $(BUILD)/route.o $(BUILD)/routes.o $(BUILD)/presort.o $(BUILD)/aggre.o $(BUILD)/engine.o $(BUILD)/batcher.o $(BUILD)/acl.o $(BUILD)/rewrite.o $(BUILD)/exchange.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -pthread $^ -L/opt/rocm/lib -lrccl -o $@

emqx_amd/libtmwork.so: emqx_amd/csrc/workload.c
	$(CC) -O2 -fPIC -shared -Wall $< -o $@ -lm

oracle/liboracle.so: oracle/o1_trie.c oracle/o3_interned.c
	$(CC) -O2 -fPIC -shared -Wall $^ -o $@ -lpthread

clean:
	rm -rf $(BUILD) emqx_amd/libtopicmatch.so emqx_amd/libtmwork.so oracle/liboracle.so

.PHONY: all clean

# Erlang NIF shim (needs OTP's erl_nif.h; not present in this image):
#   make nif ERL_INCLUDE=/usr/lib/erlang/usr/include
nif: emqx_amd/libtopicmatch.so
	@test -n "$(ERL_INCLUDE)" || (echo "set ERL_INCLUDE to the directory holding erl_nif.h" && false)
	$(CC) -O2 -fPIC -shared -I$(ERL_INCLUDE) emqx_amd/csrc/emqx_trie_nif.c -Lemqx_amd -ltopicmatch \
	  -Wl,-rpath,'$$ORIGIN' -o emqx_amd/emqx_trie_nif.so
.PHONY: nif

# micro-batcher benchmark (single-topic submits from producer threads)
tools/ubench/batcher_bench: tools/ubench/batcher_bench.cpp emqx_amd/libtopicmatch.so emqx_amd/libtmwork.so include/topicmatch.h
	$(CXX) -O2 -std=c++17 -pthread $< -Lemqx_amd -ltopicmatch -ltmwork -Wl,-rpath,'$$ORIGIN/../../emqx_amd' -o $@

# batcher driver for bench.py's batcher leg (measurement helper, ctypes)
tools/ubench/libbatchdrive.so: tools/ubench/batchdrive.cpp emqx_amd/libtopicmatch.so include/topicmatch.h
	$(CXX) -O2 -std=c++17 -fPIC -shared -pthread $< -Lemqx_amd -ltopicmatch -Wl,-rpath,'$$ORIGIN/../../emqx_amd' -o $@
