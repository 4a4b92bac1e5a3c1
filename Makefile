# Top-level build: HIP engine (gfx950) + CPU oracle.
#   make            -> openr_amd/lib/libopenr_spf.so, oracle/liboracle_spf.so
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-parameter
LIBDIR := openr_amd/lib
CSRC := openr_amd/csrc

ENGINE := $(LIBDIR)/libopenr_spf.so
ENGINE_SRCS := $(CSRC)/spf_kernels.hip $(CSRC)/spf_capi.hip
ENGINE_HDRS := $(CSRC)/spf_kernels.h include/openr_spf.h
ENGINE_OBJS := $(LIBDIR)/spf_kernels.o $(LIBDIR)/spf_capi.o

all: $(ENGINE) oracle

$(LIBDIR):
	mkdir -p $@

$(LIBDIR)/%.o: $(CSRC)/%.hip $(ENGINE_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(ENGINE): $(ENGINE_OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(ENGINE_OBJS)

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf $(LIBDIR)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
