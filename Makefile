# Build recipe for every native artefact (no cmake/ninja needed).
#   libfdf.so        HIP kernels + C ABI (the product), gfx950 only
#   liboracle.so     scalar C restatement of the reference semantics (test infrastructure)
#   libfast_avx2.so  C++ AVX2 port of the reference's fast_simd path (CPU baseline only)
#   test_cpp_api     C++ API (include/fdf.hpp) smoke binary
HIPCC ?= /opt/rocm/bin/hipcc
CC ?= gcc
CXX ?= g++
ARCH ?= gfx950

PKG := feature_detector_fast_amd
CSRC := $(PKG)/csrc
LIBFDF := $(PKG)/libfdf.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Iinclude $(EXTRA_HIPFLAGS)

all: $(LIBFDF) oracle/liboracle.so oracle/libfast_avx2.so tests/cpp/test_cpp_api

$(CSRC)/fdf_kernels.o: $(CSRC)/fdf_kernels.hip $(CSRC)/fdf_compact.h $(CSRC)/fdf_kernels.h $(CSRC)/fdf_common.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/fdf_sweep.o: $(CSRC)/fdf_sweep.hip $(CSRC)/fdf_sweep_impl.h $(CSRC)/fdf_compact.h $(CSRC)/fdf_kernels.h $(CSRC)/fdf_common.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/fdf_sweep_latency.o: $(CSRC)/fdf_sweep_latency.hip $(CSRC)/fdf_sweep_impl.h $(CSRC)/fdf_compact.h $(CSRC)/fdf_kernels.h $(CSRC)/fdf_common.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/fdf_sweep_rgb.o: $(CSRC)/fdf_sweep_rgb.hip $(CSRC)/fdf_sweep_impl.h $(CSRC)/fdf_compact.h $(CSRC)/fdf_kernels.h $(CSRC)/fdf_common.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/fdf_api.o: $(CSRC)/fdf_api.cpp $(CSRC)/fdf_kernels.h include/fdf.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/fdf_pipeline.o: $(CSRC)/fdf_pipeline.cpp include/fdf.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBFDF): $(CSRC)/fdf_kernels.o $(CSRC)/fdf_sweep.o $(CSRC)/fdf_sweep_latency.o $(CSRC)/fdf_sweep_rgb.o $(CSRC)/fdf_api.o $(CSRC)/fdf_pipeline.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

oracle/liboracle.so: oracle/fast_oracle.c oracle/fast_oracle.h
	$(CC) -O2 -std=c11 -fPIC -shared -Wall -o $@ $<

oracle/libfast_avx2.so: oracle/fast_avx2.cpp
	$(CXX) -O3 -mavx2 -std=c++17 -fPIC -shared -Wall -o $@ $< -lpthread

tests/cpp/test_cpp_api: tests/cpp/test_cpp_api.cpp include/fdf.hpp include/fdf.h $(LIBFDF)
	$(CXX) -O2 -std=c++17 -Wall -Iinclude -o $@ $< -L$(PKG) -lfdf -Wl,-rpath,'$$ORIGIN/../../$(PKG)'

# Ablation build (tools/ablate.py, tools/pmc_ablate.sh): the same library with the internal
# FDF_DEBUG_FLAGS / FDF_NSUB / FDF_LDS_BUDGET / FDF_COMPACT_TPG switches compiled in.
debug: build/libfdf_debug.so

build/libfdf_debug.so: $(CSRC)/*.hip $(CSRC)/*.cpp $(CSRC)/*.h include/fdf.h
	bash tools/build_variant.sh debug "-DFDF_DEBUG_BUILD"

clean:
	rm -f $(CSRC)/*.o $(LIBFDF) oracle/*.so tests/cpp/test_cpp_api

.PHONY: all clean debug
