# Top-level build: the gfx950 HIP library (the product), the C++ host-API
# test programs, and the test-only oracle (oracle/Makefile).
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wno-pass-failed
INC      := -Iinclude

LIB      := raikv_amd/libkvh.so
SRCS     := raikv_amd/csrc/kvh.hip raikv_amd/csrc/kvh_fixed.hip raikv_amd/csrc/kvh_varlen.hip raikv_amd/csrc/ht_pos.hip raikv_amd/csrc/crc32c.hip raikv_amd/csrc/ingest.hip raikv_amd/csrc/ht_sort.hip \
            raikv_amd/csrc/ht_refsort.hip
OBJS     := $(SRCS:.hip=.o)
HDRS     := raikv_amd/csrc/meow_dev.hpp raikv_amd/csrc/aes_tables.hpp raikv_amd/csrc/kvh_internal.hpp \
            raikv_amd/csrc/ht_pos.hpp raikv_amd/csrc/bs_prelude.hpp raikv_amd/csrc/bs_aes.hpp \
            raikv_amd/csrc/bs_meow.hpp raikv_amd/csrc/kvh_var.hpp raikv_amd/csrc/tickets.hpp include/kvh.h include/raikv_amd/key_hash.hpp

CPP_TESTS := tests/cpp/hash_test_gpu tests/cpp/bs_host_test tests/cpp/e2e_host tests/cpp/host_latency tests/cpp/paths_gpu \
             tests/cpp/kv_compat_crc tests/cpp/streams_gpu \
             tools/copy_peak tools/fetch_calib tools/scatter2_probe tools/stream_forms tools/scatter2_real \
             tools/pin_reuse_probe

KV_LIB   := raikv_amd/libkvh_kv.so

all: $(LIB) $(KV_LIB) oracle cpptests

# one object per translation unit so `make -j` compiles them in parallel
raikv_amd/csrc/%.o: raikv_amd/csrc/%.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) $(INC) -c -o $@ $<

$(LIB): $(OBJS) raikv_amd/csrc/kvh.map
	$(HIPCC) $(HIPFLAGS) -shared -Wl,--version-script=raikv_amd/csrc/kvh.map -o $@ $(OBJS)

# link-compatible kv_* Meow symbols (include/kvh_kv.h) over libkvh.so
$(KV_LIB): raikv_amd/csrc/kv_compat.cpp raikv_amd/csrc/kv_compat.map include/kvh_kv.h include/kvh.h $(LIB)
	g++ -O2 -std=c++17 -fPIC -shared $(INC) -Wl,--version-script=raikv_amd/csrc/kv_compat.map -o $@ $< \
	    -L raikv_amd -lkvh -Wl,-rpath,'$$ORIGIN'

# Research build (NOT the product): the product objects plus the research
# kernels of tools/exp/ (variants that lost their A/B, ablation builds whose
# outputs are not hashes), which register themselves behind extra
# kvh_set_tuning values (raikv_amd/csrc/kvh_internal.hpp: rt::g_exp).  Used by
# tools/*.py through KVH_LIB=tools/libkvh_exp.so; never loaded by the tests
# of the product path.
# The product sources are compiled again with -DKVH_EXPERIMENTS, which keeps
# the variants that lost their A/B (knob 7 = 7, 13, 24, 25, 44, 45, 47-50;
# knob 14 = 1-5; knob 23 = 1, 2; knob 24 = 3-5) selectable there.
EXP_LIB  := tools/libkvh_exp.so
EXP_SRCS := tools/exp/kvh_exp.hip
EXP_OBJS := $(EXP_SRCS:.hip=.o)
EXP_POBJS := $(patsubst raikv_amd/csrc/%.hip,tools/exp/obj/%.o,$(SRCS))
tools/exp/%.o: tools/exp/%.hip tools/exp/meow_exp.hpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) $(INC) -c -o $@ $<
tools/exp/obj/%.o: raikv_amd/csrc/%.hip $(HDRS)
	@mkdir -p tools/exp/obj
	$(HIPCC) $(HIPFLAGS) -DKVH_EXPERIMENTS $(INC) -c -o $@ $<
$(EXP_LIB): $(EXP_POBJS) $(EXP_OBJS) raikv_amd/csrc/kvh.map
	$(HIPCC) $(HIPFLAGS) -shared -Wl,--version-script=raikv_amd/csrc/kvh.map -o $@ $(EXP_POBJS) $(EXP_OBJS)
experiments: $(EXP_LIB)

# PROBE (not the product): the product sources with the round-4 unordered
# ticket fetches (tickets.hpp, KVH_TICKETS_UNORDERED), to show once that the
# poisoned-output test catches the chunks they drop
UNO_LIB  := tools/libkvh_unordered.so
UNO_OBJS := $(patsubst raikv_amd/csrc/%.hip,tools/uno/%.o,$(SRCS))
tools/uno/%.o: raikv_amd/csrc/%.hip $(HDRS)
	@mkdir -p tools/uno
	$(HIPCC) $(HIPFLAGS) -DKVH_TICKETS_UNORDERED $(INC) -c -o $@ $<
$(UNO_LIB): $(UNO_OBJS) raikv_amd/csrc/kvh.map
	$(HIPCC) $(HIPFLAGS) -shared -Wl,--version-script=raikv_amd/csrc/kvh.map -o $@ $(UNO_OBJS)
unordered: $(UNO_LIB)

# DEBUG BUILD (not the product): the product sources with device-side bounds
# checks (-DKVH_CHECKED; kvh_internal.hpp KVH_CHK) on the exact-order sort and
# the ingest kernels; kvh_debug_checks reads the first failed check.  Used once
# by tests/test_gpu_checked.py through KVH_LIB.
CHK_LIB  := tools/libkvh_checked.so
CHK_OBJS := $(patsubst raikv_amd/csrc/%.hip,tools/chk/%.o,$(SRCS))
tools/chk/%.o: raikv_amd/csrc/%.hip $(HDRS)
	@mkdir -p tools/chk
	$(HIPCC) $(HIPFLAGS) -DKVH_CHECKED $(INC) -c -o $@ $<
$(CHK_LIB): $(CHK_OBJS) raikv_amd/csrc/kvh.map
	$(HIPCC) $(HIPFLAGS) -shared -Wl,--version-script=raikv_amd/csrc/kvh.map -o $@ $(CHK_OBJS)
checked: $(CHK_LIB)

oracle: $(KV_LIB)
	$(MAKE) -C oracle

cpptests: $(CPP_TESTS)

tests/cpp/hash_test_gpu: tests/cpp/hash_test_gpu.cpp $(LIB) include/raikv_amd/key_hash.hpp include/kvh.h
	g++ -O2 -std=c++17 $(INC) -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ $< \
	    -L raikv_amd -lkvh -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../raikv_amd' -Wl,-rpath,/opt/rocm/lib

# the C++ API of the f1-f4 paths (key_hash.hpp) on the GPU
tests/cpp/paths_gpu: tests/cpp/paths_gpu.cpp $(LIB) include/raikv_amd/key_hash.hpp include/kvh.h
	g++ -O2 -std=c++17 $(INC) -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ $< \
	    -L raikv_amd -lkvh -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../raikv_amd' -Wl,-rpath,/opt/rocm/lib

# PCIe-inclusive host pipeline rate from a C++ host (run by bench.py --e2e)
tests/cpp/e2e_host: tests/cpp/e2e_host.cpp $(LIB) include/kvh.h
	g++ -O2 -std=c++17 $(INC) -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ $< \
	    -L raikv_amd -lkvh -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../raikv_amd' -Wl,-rpath,/opt/rocm/lib

# a C program linking only libkvh_kv.so: the CRC32C symbols of key_hash.h:8-20
tests/cpp/kv_compat_crc: tests/cpp/kv_compat_crc.c $(KV_LIB) include/kvh_kv.h
	gcc -O2 -std=c11 $(INC) -o $@ $< -L raikv_amd -lkvh_kv -Wl,-rpath,'$$ORIGIN/../../raikv_amd'

# ticket state per stream: hipStreamPerThread from several host threads, and
# launches captured into a graph and replayed on other streams
tests/cpp/streams_gpu: tests/cpp/streams_gpu.cpp $(LIB) include/kvh.h oracle
	g++ -O2 -std=c++17 $(INC) -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ $< \
	    -L raikv_amd -lkvh -L oracle -loracle -L/opt/rocm/lib -lamdhip64 -lpthread \
	    -Wl,-rpath,'$$ORIGIN/../../raikv_amd' -Wl,-rpath,'$$ORIGIN/../../oracle' -Wl,-rpath,/opt/rocm/lib

# per-call latency of the host pipelines at raikv's batch sizes, beside the
# reference CPU path (dlopen'ed from oracle/_ref at run time, test-only)
tests/cpp/host_latency: tests/cpp/host_latency.cpp $(LIB) include/kvh.h
	g++ -O2 -std=c++17 $(INC) -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ $< \
	    -L raikv_amd -lkvh -L/opt/rocm/lib -lamdhip64 -ldl \
	    -Wl,-rpath,'$$ORIGIN/../../raikv_amd' -Wl,-rpath,/opt/rocm/lib

# probe: host range registered, unregistered, unmapped and mapped again at the
# same address, then a pageable H2D copy
tools/pin_reuse_probe: tools/pin_reuse_probe.cpp $(LIB) include/kvh.h
	g++ -O2 -std=c++17 $(INC) -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ $< \
	    -L raikv_amd -lkvh -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../raikv_amd' -Wl,-rpath,/opt/rocm/lib

# measurement: the box's achievable streaming rate for bench.py's roofline
tools/copy_peak: tools/copy_peak.hip
	$(HIPCC) $(HIPFLAGS) -o $@ $<

# measurement: the streaming forms compared on one box after one settle
tools/stream_forms: tools/stream_forms.hip
	$(HIPCC) $(HIPFLAGS) -o $@ $<

# measurement: FETCH_SIZE calibration for gather access patterns
tools/fetch_calib: tools/fetch_calib.hip
	$(HIPCC) $(HIPFLAGS) -o $@ $<

# TEST ONLY: the bitsliced Meow chain run on the host against the oracle
tests/cpp/bs_host_test: tests/cpp/bs_host_test.cpp raikv_amd/csrc/bs_aes.hpp raikv_amd/csrc/bs_meow.hpp oracle
	g++ -O2 -std=c++17 -o $@ $< -Loracle -loracle -Wl,-rpath,'$$ORIGIN/../../oracle'

clean:
	rm -f $(LIB) $(KV_LIB) $(OBJS) $(CPP_TESTS) $(EXP_LIB) $(EXP_OBJS) $(EXP_POBJS) $(UNO_LIB) $(UNO_OBJS)
	$(MAKE) -C oracle clean

.PHONY: checked all oracle cpptests clean experiments unordered

# f2: the real k_tw_scatter2 under ablations: ht_sort.hip
# compiled into the probe, the product's other objects linked
PROBE_OBJS := $(filter-out raikv_amd/csrc/ht_sort.o,$(OBJS))
tools/scatter2_real: tools/scatter2_real.hip raikv_amd/csrc/ht_sort.hip $(PROBE_OBJS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) $(INC) -c -o tools/scatter2_real.o $<
	$(HIPCC) $(HIPFLAGS) -o $@ tools/scatter2_real.o $(PROBE_OBJS)

# f2 pass-2 write-pattern probe
tools/scatter2_probe: tools/scatter2_probe.hip
	$(HIPCC) $(HIPFLAGS) -Wno-unused-result -o $@ $<

# Host-code sanitizers (AddressSanitizer + UndefinedBehaviorSanitizer on the
# host side only; the device code is built as usual): the library and the C++
# programs that drive its host paths -- pipelines, ticket pool, streams,
# graphs, the C++ API -- for a run on the GPU box (tools/sessions/gpu_r5_asan.sh)
ASAN_DIR  := tools/asan
ASAN_HOST := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer
ASAN_OBJS := $(patsubst raikv_amd/csrc/%.hip,$(ASAN_DIR)/obj/%.o,$(SRCS))
ASAN_CXX  := /opt/rocm/llvm/bin/clang++ -O1 -g -std=c++17 -fsanitize=address,undefined -fno-gpu-sanitize -fno-omit-frame-pointer
ASAN_PROGS := $(ASAN_DIR)/streams_gpu $(ASAN_DIR)/e2e_host $(ASAN_DIR)/paths_gpu $(ASAN_DIR)/hash_test_gpu
$(ASAN_DIR)/obj/%.o: raikv_amd/csrc/%.hip $(HDRS)
	@mkdir -p $(ASAN_DIR)/obj
	$(HIPCC) $(HIPFLAGS) $(ASAN_HOST) $(INC) -c -o $@ $<
$(ASAN_DIR)/libkvh.so: $(ASAN_OBJS) raikv_amd/csrc/kvh.map
	$(HIPCC) $(HIPFLAGS) $(ASAN_HOST) -shared -Wl,--version-script=raikv_amd/csrc/kvh.map -o $@ $(ASAN_OBJS)
$(ASAN_DIR)/%: tests/cpp/%.cpp $(ASAN_DIR)/libkvh.so include/kvh.h include/raikv_amd/key_hash.hpp oracle
	$(ASAN_CXX) $(INC) -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ $< \
	    -L $(ASAN_DIR) -lkvh -L oracle -loracle -L/opt/rocm/lib -lamdhip64 -lpthread -ldl \
	    -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,'$$ORIGIN/../../oracle' -Wl,-rpath,/opt/rocm/lib
asan: $(ASAN_PROGS)

# ThreadSanitizer on the host code, for the multi-threaded programs (the
# streams program's host threads and the multi-pipeline host path)
TSAN_DIR  := tools/tsan
TSAN_HOST := -Xarch_host -fsanitize=thread -Xarch_host -fno-omit-frame-pointer
TSAN_OBJS := $(patsubst raikv_amd/csrc/%.hip,$(TSAN_DIR)/obj/%.o,$(SRCS))
TSAN_CXX  := /opt/rocm/llvm/bin/clang++ -O1 -g -std=c++17 -fsanitize=thread -fno-gpu-sanitize -fno-omit-frame-pointer
$(TSAN_DIR)/obj/%.o: raikv_amd/csrc/%.hip $(HDRS)
	@mkdir -p $(TSAN_DIR)/obj
	$(HIPCC) $(HIPFLAGS) $(TSAN_HOST) $(INC) -c -o $@ $<
$(TSAN_DIR)/libkvh.so: $(TSAN_OBJS) raikv_amd/csrc/kvh.map
	$(HIPCC) $(HIPFLAGS) $(TSAN_HOST) -shared -Wl,--version-script=raikv_amd/csrc/kvh.map -o $@ $(TSAN_OBJS)
$(TSAN_DIR)/%: tests/cpp/%.cpp $(TSAN_DIR)/libkvh.so include/kvh.h oracle
	$(TSAN_CXX) $(INC) -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o $@ $< \
	    -L $(TSAN_DIR) -lkvh -L oracle -loracle -L/opt/rocm/lib -lamdhip64 -lpthread -ldl \
	    -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,'$$ORIGIN/../../oracle' -Wl,-rpath,/opt/rocm/lib
tsan: $(TSAN_DIR)/streams_gpu $(TSAN_DIR)/e2e_host
