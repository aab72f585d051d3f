# Build for MI355X (gfx950) only.  Outputs stay in-tree so they travel to the GPU box.
#   make          -> qec_ldpc_amd/libqecldpc.so, oracle/liboracle.so, tools/qec_ldpc (CLI)
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
# IEEE fp32 exactly as written: no contraction, no fast-math, denormals preserved.
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wall -Wno-unused-function
CSRC     := qec_ldpc_amd/csrc
OBJ      := build/obj
LIB      := qec_ldpc_amd/libqecldpc.so
OBJS     := $(OBJ)/bp_decode.o $(OBJ)/bp_decode_p61.o $(OBJ)/bp_decode_phase.o $(OBJ)/bp_sparse.o $(OBJ)/schedule.o $(OBJ)/triage.o $(OBJ)/montecarlo.o $(OBJ)/code_model.o $(OBJ)/cpu_engine.o $(OBJ)/capi.o
HDRS     := include/qec_ldpc.h include/HostDeviceArray.h $(CSRC)/qec_internal.h $(CSRC)/qec_device.h $(CSRC)/qec_mc.h $(CSRC)/qec_launch.h
# build id: hash of every library source and this Makefile (identical for every rebuild of one tree);
# profiles/pmc_*.json carry it and bench.py uses a profile only with the library it was taken on
SRCS     := $(sort $(wildcard $(CSRC)/*.hip $(CSRC)/*.cpp $(CSRC)/*.h)) include/qec_ldpc.h include/HostDeviceArray.h Makefile
BUILD_ID := $(shell cat $(SRCS) | sha256sum | cut -c1-16)

all: $(LIB) oracle tools/qec_ldpc tools/getstats_check

$(OBJ):
	mkdir -p $(OBJ)

$(OBJ)/bp_decode.o: $(CSRC)/bp_decode.hip $(HDRS) | $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the P61 reference/fixed-stop kernels under the iterative-minreg scheduler (bp_decode.hip, TuneP61)
$(OBJ)/bp_decode_p61.o: $(CSRC)/bp_decode_p61.hip $(CSRC)/bp_decode.hip $(HDRS) | $(OBJ)
	$(HIPCC) $(HIPFLAGS) -mllvm -amdgpu-sched-strategy=iterative-minreg -c $< -o $@

# the instrumented kernels of QEC_OPT_PHASE_STATS (bp_decode.hip, QEC_PHASE_STATS)
$(OBJ)/bp_decode_phase.o: $(CSRC)/bp_decode_phase.hip $(CSRC)/bp_decode.hip $(HDRS) | $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/bp_sparse.o: $(CSRC)/bp_sparse.hip $(HDRS) | $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/schedule.o: $(CSRC)/schedule.hip $(HDRS) | $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/triage.o: $(CSRC)/triage.hip $(HDRS) | $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/montecarlo.o: $(CSRC)/montecarlo.hip $(HDRS) | $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/code_model.o: $(CSRC)/code_model.cpp $(HDRS) | $(OBJ)
	$(HIPCC) $(HIPFLAGS) -x c++ -c $< -o $@

$(OBJ)/cpu_engine.o: $(CSRC)/cpu_engine.cpp $(HDRS) | $(OBJ)
	$(HIPCC) $(HIPFLAGS) -x c++ -c $< -o $@

$(OBJ)/capi.o: $(SRCS) | $(OBJ)
	$(HIPCC) $(HIPFLAGS) -DQEC_BUILD_ID='"$(BUILD_ID)"' -x hip -c $(CSRC)/capi.cpp -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -Wl,--no-undefined

# main.cu's Monte-Carlo driver on the GPU engine (caller side, tools/qec_ldpc_main.cpp)
tools/qec_ldpc: tools/qec_ldpc_main.cpp include/*.h $(LIB)
	$(HIPCC) -O2 -std=c++17 -Iinclude -o $@ $< -Lqec_ldpc_amd -lqecldpc -Wl,-rpath,'$$ORIGIN/../qec_ldpc_amd'

# DecoderGPU::GetStats vs GetStatistics through the C++ interface (tests/test_gpu_kat.py)
tools/getstats_check: tools/getstats_check.cpp include/*.h $(LIB)
	$(HIPCC) -O2 -std=c++17 -Iinclude -o $@ $< -Lqec_ldpc_amd -lqecldpc -Wl,-rpath,'$$ORIGIN/../qec_ldpc_amd'

oracle:
	$(MAKE) -s -C oracle

# Host-code race check under ThreadSanitizer: the product's code model and
# the oracle (without OpenMP) driven from 8 threads over shared code objects; tests/test_tsan.py
TSAN_BIN := build/tsan/tsan_check
tsan: $(TSAN_BIN)
$(TSAN_BIN): tests/tsan/tsan_check.cpp $(CSRC)/code_model.cpp oracle/qec_oracle.c $(CSRC)/qec_internal.h include/qec_ldpc.h
	mkdir -p build/tsan
	gcc -O1 -g -fsanitize=thread -ffp-contract=off -fPIC -c oracle/qec_oracle.c -o build/tsan/qec_oracle.o
	g++ -O1 -g -std=c++17 -fsanitize=thread -c $(CSRC)/code_model.cpp -o build/tsan/code_model.o
	g++ -O1 -g -std=c++17 -fsanitize=thread tests/tsan/tsan_check.cpp build/tsan/code_model.o build/tsan/qec_oracle.o -o $@ -lpthread

clean:
	rm -rf build $(LIB) tools/qec_ldpc tools/getstats_check
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean tsan
