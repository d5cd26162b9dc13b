# Build of every native artefact.  Outputs stay in-tree so they travel with
# the gpurun snapshot (they are git-ignored).
#   dcvc_amd/lib/libdcvc_rans.so  host rANS coder (C ABI: include/dcvc_rans.h)
#   dcvc_amd/lib/libdcvc_hip.so   gfx950 HIP kernels (C ABI: include/dcvc_hip.h)
#   oracle/_build/liboracle_rans.so  test-only C restatement of the coder
#   oracle/_ref/                  test-only build of the reference's own
#                                  ops.cpp (only when /root/reference exists)
HIPCC    ?= /opt/rocm/bin/hipcc
# -fno-slp-vectorize: no packed-f32 VALU instructions in the kernels
# (scripts/check_isa.sh explains why and enforces it)
HIPFLAGS ?= -fno-slp-vectorize
# make XCONV_DBG=1: xconv.hip with its timing-ablation switches (diagnostics only)
ifdef XCONV_DBG
HIPFLAGS += -DXCONV_DBG
endif
CXX      ?= g++
CC       ?= gcc
ARCH     ?= gfx950
PYTHON   ?= python3

LIB      := dcvc_amd/lib
HIP_SRCS := $(wildcard dcvc_amd/csrc/hip/*.hip)
HIP_HDRS := $(wildcard dcvc_amd/csrc/hip/*.h) include/dcvc_hip.h
HIP_OBJS := $(patsubst dcvc_amd/csrc/hip/%.hip,build/hip/%.o,$(HIP_SRCS))

REF      := /root/reference
PYBIND   := $(shell $(PYTHON) -c "import pybind11;print(pybind11.get_include())" 2>/dev/null)
PYINC    := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_paths()['include'])" 2>/dev/null)
PYEXT    := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))" 2>/dev/null)

all: rans hip oracle

rans: $(LIB)/libdcvc_rans.so
hip: $(LIB)/libdcvc_hip.so
oracle: oracle/_build/liboracle_rans.so ref

$(LIB)/libdcvc_rans.so: dcvc_amd/csrc/rans/dcvc_rans.cpp include/dcvc_rans.h
	@mkdir -p $(LIB)
	$(CXX) -std=c++17 -O3 -march=x86-64-v2 -fPIC -shared -pthread -Wall -Wextra -o $@ $<

build/hip/%.o: dcvc_amd/csrc/hip/%.hip $(HIP_HDRS)
	@mkdir -p build/hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall $(HIPFLAGS) -c -o $@ $<

# check_isa.sh: no packed-f32 VALU, no scratch in the split kernels;
# check_xconv_vmcnt.py: every xconv3_kernel instantiation issues exactly the
# vector-memory instructions its exact vmcnt waits count, and so do
# wconv3_kernel's DMA wave and the streamed sffn_kernels (the library is
# linked to a temporary name first and only kept if the check passes)
$(LIB)/libdcvc_hip.so: $(HIP_OBJS) scripts/check_isa.sh scripts/check_xconv_vmcnt.py
	@mkdir -p $(LIB)
	bash scripts/check_isa.sh $(HIP_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@.tmp $(HIP_OBJS)
	$(PYTHON) scripts/check_xconv_vmcnt.py $@.tmp build/hip/xconv.o || { rm -f $@.tmp; exit 1; }
	$(PYTHON) scripts/check_xconv_vmcnt.py $@.tmp build/hip/wconv.o || { rm -f $@.tmp; exit 1; }
	$(PYTHON) scripts/check_xconv_vmcnt.py $@.tmp build/hip/sffn.o || { rm -f $@.tmp; exit 1; }
	mv $@.tmp $@

oracle/_build/liboracle_rans.so: oracle/rans_oracle.c
	@mkdir -p oracle/_build
	$(CC) -O2 -fPIC -shared -Wall -o $@ $< -lm

# The reference's own PMF->CDF quantizer, compiled from its single source file
# (DCVC-DC/src/cpp/ops/ops.cpp) against the installed pybind11.  The rANS
# sources are NOT built: they need ryg_rans' rans64.h, which is not on disk.
ref:
	@if [ -f $(REF)/DCVC-DC/src/cpp/ops/ops.cpp ] && [ -n "$(PYBIND)" ]; then \
	  mkdir -p oracle/_ref; \
	  if [ ! -f oracle/_ref/MLCodec_CXX$(PYEXT) ] || [ $(REF)/DCVC-DC/src/cpp/ops/ops.cpp -nt oracle/_ref/MLCodec_CXX$(PYEXT) ]; then \
	    echo "building oracle/_ref/MLCodec_CXX$(PYEXT) from reference ops.cpp"; \
	    $(CXX) -std=c++17 -O2 -fPIC -shared -I$(PYBIND) -I$(PYINC) \
	      -o oracle/_ref/MLCodec_CXX$(PYEXT) $(REF)/DCVC-DC/src/cpp/ops/ops.cpp; \
	  fi; \
	else echo "reference not present: skipping oracle/_ref"; fi

clean:
	rm -rf build $(LIB) oracle/_build oracle/_ref

.PHONY: all rans hip oracle ref clean
