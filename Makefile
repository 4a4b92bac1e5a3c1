# Top-level build: HIP engine (gfx950) + C++ host mirror + CPU oracle + C++ tests.
#   make            -> openr_amd/lib/libopenr_spf.so, openr_amd/lib/libopenr_decision.so,
#                      oracle/liboracle_spf.so, tests/cpp/build/{linkstate,decision}_test
#
# Build provenance: every library / test binary embeds a build id
#   "<sha256/16 of its sources> <source files>"
# (openr_spf_build_id / openr_decision_build_id / "build-id:" line of the test binaries).
# openr_amd/engine.py and tests/ recompute the hash from the tree they run in and refuse
# a binary built from other sources, so a GPU run cannot silently use a stale .so.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-parameter \
            -mllvm -amdgpu-atomic-optimizer-strategy=None
LIBDIR := openr_amd/lib
CSRC := openr_amd/csrc

ENGINE := $(LIBDIR)/libopenr_spf.so
ENGINE_SRCS := $(CSRC)/spf_kernels.hip $(CSRC)/spf_bfs.hip $(CSRC)/spf_bfs_lvl.hip $(CSRC)/spf_sweep.hip $(CSRC)/spf_fringe.hip $(CSRC)/spf_rounds.hip $(CSRC)/spf_ksp.hip $(CSRC)/spf_update.hip $(CSRC)/spf_exact.hip $(CSRC)/spf_capi.hip
ENGINE_HDRS := $(CSRC)/spf_kernels.h $(CSRC)/spf_device.h $(CSRC)/spf_bfs_common.h include/openr_spf.h
ENGINE_OBJS := $(patsubst $(CSRC)/%.hip,$(LIBDIR)/%.o,$(ENGINE_SRCS))

HOST := $(LIBDIR)/libopenr_decision.so
HOST_SRCS := $(CSRC)/host/LinkState.cpp $(CSRC)/host/Decision.cpp $(CSRC)/host/AdjDbCodec.cpp $(CSRC)/host/adjdb_capi.cpp $(CSRC)/host/wan_gen.cpp
HOST_HDRS := $(CSRC)/host/LinkState.h $(CSRC)/host/Decision.h $(CSRC)/host/HostParallel.h $(CSRC)/host/AdjDbCodec.h include/openr_spf.h include/openr_adjdb.h include/openr_topogen.h include/openr_routes.h
CXX ?= g++
CC ?= gcc
CXXFLAGS ?= -O2 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter
CPPTEST := tests/cpp/build/linkstate_test
DECTEST := tests/cpp/build/decision_test
DECBENCH := tests/cpp/build/decision_bench
CPPTEST_SRCS := tests/cpp/linkstate_test.cpp tests/cpp/harness.h oracle/spf_oracle.c oracle/spf_oracle.h
DECTEST_SRCS := tests/cpp/decision_test.cpp tests/cpp/harness.h openr_amd/csrc/host/HostParallel.h oracle/spf_oracle.c oracle/spf_oracle.h

# "<hash> <files>" of a file list (the same recipe as openr_amd/engine.py:source_hash)
build_id = $$(cat $(1) | sha256sum | cut -c1-16) $(1)

all: $(ENGINE) $(HOST) oracle $(CPPTEST) $(DECTEST) $(DECBENCH)

$(LIBDIR):
	mkdir -p $@

$(LIBDIR)/%.o: $(CSRC)/%.hip $(ENGINE_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(ENGINE): $(ENGINE_OBJS) $(ENGINE_SRCS) $(ENGINE_HDRS)
	printf 'const char* openr_spf_build_id(void) { return "%s"; }\n' "$(call build_id,$(ENGINE_SRCS) $(ENGINE_HDRS))" > $(LIBDIR)/spf_build_id.c
	$(CC) -O2 -fPIC -c $(LIBDIR)/spf_build_id.c -o $(LIBDIR)/spf_build_id.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(ENGINE_OBJS) $(LIBDIR)/spf_build_id.o

# C++ host mirror of openr::LinkState over the C-ABI (links the engine)
$(HOST): $(HOST_SRCS) $(HOST_HDRS) $(ENGINE)
	$(CXX) $(CXXFLAGS) -shared -o $@ $(HOST_SRCS) \
	  -DOPENR_DECISION_BUILD_ID="\"$(call build_id,$(HOST_SRCS) $(HOST_HDRS))\"" \
	  -L$(LIBDIR) -lopenr_spf -pthread -Wl,-rpath,'$$ORIGIN'

# C++ tests of the host mirror (oracle linked as the checker)
$(CPPTEST): $(CPPTEST_SRCS) $(HOST)
	mkdir -p tests/cpp/build
	$(CC) -O2 -std=c11 -fPIC -c oracle/spf_oracle.c -o tests/cpp/build/spf_oracle.o
	$(CXX) $(CXXFLAGS) -o $@ tests/cpp/linkstate_test.cpp tests/cpp/build/spf_oracle.o \
	  -DOPENR_TEST_BUILD_ID="\"$(call build_id,$(CPPTEST_SRCS))\"" \
	  -L$(LIBDIR) -lopenr_decision -lopenr_spf -pthread -Wl,-rpath,'$$ORIGIN/../../../$(LIBDIR)'

# C++ tests of the SpfSolver / RibPolicy mirror (oracle linked as the checker)
$(DECTEST): $(DECTEST_SRCS) $(HOST)
	mkdir -p tests/cpp/build
	$(CC) -O2 -std=c11 -fPIC -c oracle/spf_oracle.c -o tests/cpp/build/spf_oracle_d.o
	$(CXX) $(CXXFLAGS) -o $@ tests/cpp/decision_test.cpp tests/cpp/build/spf_oracle_d.o \
	  -DOPENR_TEST_BUILD_ID="\"$(call build_id,$(DECTEST_SRCS))\"" \
	  -L$(LIBDIR) -lopenr_decision -lopenr_spf -pthread -Wl,-rpath,'$$ORIGIN/../../../$(LIBDIR)'

# DecisionBenchmark through the drop-in (bench.py --workload decision); links the oracle as
# the checker and the faithful-cost CPU baseline
$(DECBENCH): tests/cpp/decision_bench.cpp $(HOST) oracle
	mkdir -p tests/cpp/build
	$(CXX) $(CXXFLAGS) -o $@ tests/cpp/decision_bench.cpp oracle/spf_oracle.o oracle/spf_faithful.o \
	  -L$(LIBDIR) -lopenr_decision -lopenr_spf -pthread -Wl,-rpath,'$$ORIGIN/../../../$(LIBDIR)'

# Host-side profile of the route build (test infrastructure): the host sources, the
# DecisionBenchmark harness and the CPU oracle standing in for the GPU engine
# (tests/cpp/cpu_engine_stub.cpp), compiled with -pg. Not part of `all`; never shipped.
host_profile: oracle
	mkdir -p tests/cpp/build
	$(CXX) -O2 -g -pg -std=c++17 -o tests/cpp/build/host_profile tests/cpp/decision_bench.cpp tests/cpp/cpu_engine_stub.cpp \
	  $(filter %.cpp,$(HOST_SRCS)) oracle/spf_oracle.o oracle/spf_faithful.o -pthread

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf $(LIBDIR) tests/cpp/build
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean host_profile
