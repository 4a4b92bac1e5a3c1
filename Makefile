# Top-level build: HIP engine (gfx950) + CPU oracle.
#   make            -> openr_amd/lib/libopenr_spf.so, oracle/liboracle_spf.so
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-parameter \
            -mllvm -amdgpu-atomic-optimizer-strategy=None
LIBDIR := openr_amd/lib
CSRC := openr_amd/csrc

ENGINE := $(LIBDIR)/libopenr_spf.so
ENGINE_SRCS := $(CSRC)/spf_kernels.hip $(CSRC)/spf_bfs.hip $(CSRC)/spf_bfs_lvl.hip $(CSRC)/spf_sweep.hip $(CSRC)/spf_fringe.hip $(CSRC)/spf_rounds.hip $(CSRC)/spf_ksp.hip $(CSRC)/spf_update.hip $(CSRC)/spf_capi.hip
ENGINE_HDRS := $(CSRC)/spf_kernels.h $(CSRC)/spf_device.h $(CSRC)/spf_bfs_common.h include/openr_spf.h
ENGINE_OBJS := $(LIBDIR)/spf_kernels.o $(LIBDIR)/spf_bfs.o $(LIBDIR)/spf_bfs_lvl.o $(LIBDIR)/spf_sweep.o $(LIBDIR)/spf_fringe.o $(LIBDIR)/spf_rounds.o $(LIBDIR)/spf_ksp.o $(LIBDIR)/spf_update.o $(LIBDIR)/spf_capi.o

HOST := $(LIBDIR)/libopenr_decision.so
HOST_SRCS := $(CSRC)/host/LinkState.cpp $(CSRC)/host/Decision.cpp $(CSRC)/host/AdjDbCodec.cpp $(CSRC)/host/adjdb_capi.cpp
HOST_HDRS := $(CSRC)/host/LinkState.h $(CSRC)/host/Decision.h $(CSRC)/host/AdjDbCodec.h include/openr_spf.h include/openr_adjdb.h
CXX ?= g++
CC ?= gcc
CXXFLAGS ?= -O2 -g -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter
CPPTEST := tests/cpp/build/linkstate_test
DECTEST := tests/cpp/build/decision_test

all: $(ENGINE) $(HOST) oracle $(CPPTEST) $(DECTEST)

$(LIBDIR):
	mkdir -p $@

$(LIBDIR)/%.o: $(CSRC)/%.hip $(ENGINE_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(ENGINE): $(ENGINE_OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(ENGINE_OBJS)

# C++ host mirror of openr::LinkState over the C-ABI (links the engine)
$(HOST): $(HOST_SRCS) $(HOST_HDRS) $(ENGINE)
	$(CXX) $(CXXFLAGS) -shared -o $@ $(HOST_SRCS) -L$(LIBDIR) -lopenr_spf -Wl,-rpath,'$$ORIGIN'

# C++ tests of the host mirror (oracle linked as the checker)
$(CPPTEST): tests/cpp/linkstate_test.cpp tests/cpp/harness.h $(HOST) oracle/spf_oracle.c oracle/spf_oracle.h
	mkdir -p tests/cpp/build
	$(CC) -O2 -g -std=c11 -c oracle/spf_oracle.c -o tests/cpp/build/spf_oracle.o
	$(CXX) $(CXXFLAGS) -o $@ tests/cpp/linkstate_test.cpp tests/cpp/build/spf_oracle.o \
	  -L$(LIBDIR) -lopenr_decision -lopenr_spf -pthread -Wl,-rpath,'$$ORIGIN/../../../$(LIBDIR)'

# C++ tests of the SpfSolver / RibPolicy mirror
$(DECTEST): tests/cpp/decision_test.cpp tests/cpp/harness.h $(HOST)
	mkdir -p tests/cpp/build
	$(CXX) $(CXXFLAGS) -o $@ tests/cpp/decision_test.cpp \
	  -L$(LIBDIR) -lopenr_decision -lopenr_spf -pthread -Wl,-rpath,'$$ORIGIN/../../../$(LIBDIR)'

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf $(LIBDIR) tests/cpp/build
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
