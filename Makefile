# Build for the MI355X path tracer.  Targets:
#   make            host lib + HIP lib + CLI + oracle (everything __graft_entry__.build() needs)
#   make hip        cuda_raytracing_amd/lib/librt_hip.so    (hipcc, gfx950)
#   make host       cuda_raytracing_amd/lib/librt_host.so   (g++)
#   make oracle     oracle/_build/liboracle_rt.so           (gcc + OpenMP; test infrastructure)
#   make cli        bin/raytracing                          (reference CLI surface)
#   make kat        regenerate tests/golden/rng_kat.json from rocRAND

ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
ARCH      ?= gfx950
CXX       ?= g++
CC        ?= gcc

LIBDIR    := cuda_raytracing_amd/lib
CSRC      := cuda_raytracing_amd/csrc
INC       := -Iinclude -I$(CSRC)

# No FP contraction anywhere on the path: parity with the oracle is bit-exact.
HOST_FLAGS := -O2 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wextra
HIP_FLAGS  := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -fno-fast-math \
              -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-rdc -fno-slp-vectorize -Wall
ORACLE_FLAGS := -O2 -std=c11 -fPIC -ffp-contract=off -fno-fast-math -fopenmp -Wall -Wextra

HOST_SRC := $(CSRC)/host/rt_host.cpp $(CSRC)/host/image_load.cpp $(CSRC)/host/image_jpeg.cpp \
            $(CSRC)/host/image_png.cpp
HIP_SRC  := $(CSRC)/rt_device.hip $(CSRC)/rt_capi.cpp $(CSRC)/scene_compile.cpp $(CSRC)/xorwow_jump.cpp \
            $(CSRC)/sphere_accel.cpp $(CSRC)/mixed_accel.cpp \
            $(CSRC)/scene_codegen.cpp $(CSRC)/rt_jit.cpp $(CSRC)/rt_multi.cpp $(CSRC)/code_object.cpp
HIP_HDR  := $(wildcard $(CSRC)/*.h) $(CSRC)/device/rt_layout.h $(CSRC)/device/rt_body.h \
            $(CSRC)/device/embedded_headers.inc include/rt_render.h include/rt_ref_layout.h

# Each library records the hash of the sources it was built from (rt_hip_build_hash / rt_host_build_hash); the Python
# binding recomputes it over the same files and refuses a library that does not match the tree, so a stale prebuilt
# .so can never be what a test, smoke() or bench.py runs (build() is the only producer of the libraries they load)
HIP_STAMP_SRC  := $(sort $(HIP_SRC) $(filter-out $(CSRC)/device/embedded_headers.inc,$(HIP_HDR)) $(CSRC)/jitc/rt_jitc.cpp)
HOST_STAMP_SRC := $(sort $(HOST_SRC) $(CSRC)/host/glibc_rand.h $(CSRC)/host/image_decoders.h include/rt_host.h \
                    include/rt_ref_layout.h include/rt_render.h)
stamp = -DRT_SOURCE_HASH='"$(shell cat $(1) | sha256sum | cut -c1-16)"' -DRT_SOURCE_FILES='"$(1)"'

all: host hip oracle cli ref

host: $(LIBDIR)/librt_host.so
hip: $(LIBDIR)/librt_hip.so $(LIBDIR)/rt_jitc
oracle: oracle/_build/liboracle_rt.so
cli: bin/raytracing

$(LIBDIR)/librt_host.so: $(HOST_SRC) $(CSRC)/host/glibc_rand.h $(CSRC)/host/image_decoders.h include/rt_host.h include/rt_ref_layout.h include/rt_render.h
	@mkdir -p $(LIBDIR)
	$(CXX) $(HOST_FLAGS) $(INC) $(call stamp,$(HOST_STAMP_SRC)) -shared $(HOST_SRC) -o $@

# device headers embedded as text for the run-time (hipRTC) scene-specialised kernels
$(CSRC)/device/embedded_headers.inc: $(CSRC)/device/rt_layout.h $(CSRC)/device/rt_body.h tools/embed_headers.py
	python3 tools/embed_headers.py $@ kEmbedLayout=$(CSRC)/device/rt_layout.h kEmbedBody=$(CSRC)/device/rt_body.h

$(LIBDIR)/librt_hip.so: $(HIP_SRC) $(HIP_HDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIP_FLAGS) $(INC) $(call stamp,$(HIP_STAMP_SRC)) -shared $(HIP_SRC) -o $@ -L$(ROCM)/lib -lhiprtc -ldl

# the run-time kernels' compiler process (rt_jit.cpp): /opt/rocm's hipRTC, whatever the calling process loaded
$(LIBDIR)/rt_jitc: $(CSRC)/jitc/rt_jitc.cpp
	@mkdir -p $(LIBDIR)
	$(CXX) -O2 -std=c++17 -Wall -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include $< -o $@ -L$(ROCM)/lib -lhiprtc \
	  -Wl,-rpath,$(ROCM)/lib

oracle/_build/liboracle_rt.so: oracle/oracle_rt.c include/rt_render.h include/rt_ref_layout.h
	@mkdir -p oracle/_build
	$(CC) $(ORACLE_FLAGS) -Iinclude -shared oracle/oracle_rt.c -o $@ -lm

bin/raytracing: $(CSRC)/host/cli.cpp $(LIBDIR)/librt_host.so $(LIBDIR)/librt_hip.so include/rt_host.h
	@mkdir -p bin
	$(CXX) $(HOST_FLAGS) $(INC) $(CSRC)/host/cli.cpp -o $@ -L$(LIBDIR) -lrt_host -lrt_hip \
	  -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'

# reference-side checker (test infrastructure): the reference's stb_image compiled where it lies, only
# when the reference tree is present (not on the GPU box); output only into oracle/_ref/
REF_INC ?= /root/reference/include
CLANGXX ?= $(ROCM)/lib/llvm/bin/clang++
ref:
	@if [ -f $(REF_INC)/stb_image.h ]; then mkdir -p oracle/_ref && \
	  $(CXX) -O2 -fPIC -shared -w -I$(REF_INC) oracle/stbi_ref.cpp -o oracle/_ref/libstbi_ref.so && \
	  $(CLANGXX) -O2 -fPIC -shared -w -ftrivial-auto-var-init=zero -DRT_STBI_FILL=0 -I$(REF_INC) \
	    oracle/stbi_ref.cpp -o oracle/_ref/libstbi_ref_zero.so && \
	  $(CLANGXX) -O2 -fPIC -shared -w -ftrivial-auto-var-init=pattern -DRT_STBI_FILL=0xA5 -I$(REF_INC) \
	    oracle/stbi_ref.cpp -o oracle/_ref/libstbi_ref_pattern.so; \
	  else echo "ref: $(REF_INC)/stb_image.h not present, skipping oracle/_ref"; fi

kat:
	$(CXX) -O1 -std=c++17 -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include oracle/kat/gen_rocrand_kat.cpp \
	  -o oracle/_build/gen_rocrand_kat -L$(ROCM)/lib -lamdhip64 -Wno-deprecated-declarations
	oracle/_build/gen_rocrand_kat > tests/golden/rng_kat.json

clean:
	rm -rf $(LIBDIR)/*.so $(LIBDIR)/rt_jitc oracle/_build bin

.PHONY: all host hip oracle cli ref kat clean
