# Build of the MI355X ray-trace path (no cmake needed; outputs stay in-tree so they travel
# to the GPU box with the snapshot).
#   make            -> ray_tracying_amd/lib/librt_hip.so  (hipcc, gfx950 kernels + C ABI)
#                      ray_tracying_amd/lib/librt_host.so (g++, scene loader / BVH / PPM)
#                      ray_tracying_amd/bin/raytracer     (drop-in CLI)
#                      oracle/liboracle.so, oracle/oracle_cli (CPU restatement, tests only)
#   make ref        -> oracle/_ref/{Raytracer,ref_driver} from /root/reference (tests only)
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
# exact IEEE binary32: no FMA contraction, correctly rounded div/sqrt on the device.
# -fno-slp-vectorize: the SLP vectoriser paired scalar f32 ops into v_pk_add/v_pk_mul and built
# the register pairs with moves (trace kernel 125 -> 84 VGPRs without it, 5 waves/SIMD fit;
# headline +4 %, C4 +7 %, round 2 A/B).  The explicit f32x2 culling fma stays packed.
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -fPIC -Wno-unused-result
CXXFLAGS := -O2 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-function
LIB := ray_tracying_amd/lib
BIN := ray_tracying_amd/bin
SRC := ray_tracying_amd/csrc
COMMON_H := $(SRC)/common/rt_powf.h $(SRC)/common/glibc_powf_data.h include/rt_hip.h

all: $(LIB)/librt_hip.so $(LIB)/librt_host.so $(LIB)/librt_comm.so $(BIN)/raytracer oracle

$(LIB)/librt_hip.so: $(SRC)/hip/rt_hip.hip $(SRC)/hip/rt_device.h $(COMMON_H)
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -shared $(SRC)/hip/rt_hip.hip -o $@

HOST_SRC := $(SRC)/host/json_dom.cpp $(SRC)/host/scene.cpp $(SRC)/host/bvh_wide.cpp $(SRC)/host/rt_host_api.cpp
$(LIB)/librt_host.so: $(HOST_SRC) $(SRC)/host/json_dom.hpp $(SRC)/host/scene.hpp include/rt_host.h $(COMMON_H) $(LIB)/librt_hip.so
	$(CXX) $(CXXFLAGS) -shared $(HOST_SRC) -o $@ -L$(LIB) -lrt_hip -Wl,-rpath,'$$ORIGIN'

# RCCL collectives (librccl from ROCm) for the multi-GPU tile gather
$(LIB)/librt_comm.so: $(SRC)/comm/rt_comm.cpp include/rt_comm.h include/rt_hip.h
	@mkdir -p $(LIB)
	$(HIPCC) -O2 -std=c++17 -fPIC -shared $(SRC)/comm/rt_comm.cpp -o $@ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

$(BIN)/raytracer: $(SRC)/host/main.cpp $(LIB)/librt_host.so $(LIB)/librt_comm.so include/rt_comm.h
	@mkdir -p $(BIN)
	$(CXX) $(CXXFLAGS) $(SRC)/host/main.cpp -o $@ -L$(LIB) -lrt_host -lrt_comm -lrt_hip -lpthread -Wl,-rpath,'$$ORIGIN/../lib'

# A/B build of the HIP library with extra defines (or another source, VSRC: e.g. the previous
# commit's rt_hip.hip saved beside it) into ray_tracying_amd/lib_$(V)/ (diagnostic; select it
# at run time with RT_LIB_DIR): make variant V=w5 VDEFS=-DRT_TRACE_WAVES=5
VSRC ?= $(SRC)/hip/rt_hip.hip
variant: $(LIB)/librt_host.so
	@mkdir -p ray_tracying_amd/lib_$(V)
	$(HIPCC) $(HIPFLAGS) $(VDEFS) -shared $(VSRC) -o ray_tracying_amd/lib_$(V)/librt_hip.so
	cp $(LIB)/librt_host.so $(LIB)/librt_comm.so ray_tracying_amd/lib_$(V)/

# Host code and oracle under AddressSanitizer + UndefinedBehaviorSanitizer (host only: the
# GPU pool runs no sanitizers on device code).  Run the CPU suite against them with
#   make asan && LD_PRELOAD="$$(g++ -print-file-name=libasan.so) $$(g++ -print-file-name=libstdc++.so)" ASAN_OPTIONS=detect_leaks=0 \
#   RT_LIB_DIR=ray_tracying_amd/lib_asan ORACLE_SO=oracle/_asan/liboracle.so python -m pytest tests -m "not gpu"
SANFLAGS := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1
asan: $(LIB)/librt_hip.so $(LIB)/librt_comm.so
	@mkdir -p ray_tracying_amd/lib_asan
	$(CXX) $(CXXFLAGS) $(SANFLAGS) -shared $(HOST_SRC) -o ray_tracying_amd/lib_asan/librt_host.so -L$(LIB) -lrt_hip -Wl,-rpath,'$$ORIGIN' -pthread
	cp $(LIB)/librt_hip.so $(LIB)/librt_comm.so ray_tracying_amd/lib_asan/
	$(MAKE) -C oracle asan SANFLAGS="$(SANFLAGS)"

# The counter-measured VALU peak (tools/measure_r03.sh runs it under rocprofv3 --pmc): built
# with the device code's own flags -- with the SLP vectoriser on, the mixed int / convert /
# fp32 kind becomes v_pk_add_f32 + moves and issues at 1.18 instead of 1.73 per CU-cycle
ubench: tools/bin/ubench_valu
tools/bin/ubench_valu: tools/ubench_valu.hip
	@mkdir -p tools/bin
	$(HIPCC) $(filter-out -fPIC,$(HIPFLAGS)) tools/ubench_valu.hip -o $@

oracle:
	$(MAKE) -C oracle all

ref:
	$(MAKE) -C oracle ref

clean:
	rm -rf $(LIB) $(BIN)
	$(MAKE) -C oracle clean

.PHONY: all oracle ref clean variant asan ubench
