# Build everything in-tree (the built .so files travel to the GPU box with the snapshot).
#   make            -> product: xalm_amd/lib/libxalm_hip.so, libxalm_host.so, xalm_amd/bin/xalm
#                      test infrastructure: oracle/lib/liboracle.so
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
CC ?= gcc
ARCH ?= gfx950

HIPFLAGS := -O3 --offload-arch=$(ARCH) -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result $(HIPFLAGS_EXTRA)
HOSTFLAGS := -O2 -std=c++17 -fPIC -Wall -Wextra

LIB := xalm_amd/lib
BIN := xalm_amd/bin
HIP_SRC := xalm_amd/csrc/xalm_hip.hip
HIP_HDR := $(wildcard xalm_amd/csrc/*.h) include/xalm_hip.h
HOST_SRC := $(wildcard xalm_amd/host/*.cpp)
HOST_HDR := $(wildcard xalm_amd/host/*.h) include/xalm_hip.h include/xalm_host.h

.PHONY: all product oracle clean
all: product oracle
ifneq ($(HOST_SRC),)
product: $(LIB)/libxalm_hip.so $(LIB)/libxalm_host.so $(BIN)/xalm
else
product: $(LIB)/libxalm_hip.so
endif
oracle:
	$(MAKE) -C oracle

# the fused attention + Wo kernel is instantiated per Wo dtype in its own objects (parallel build)
OBJ := xalm_amd/build
PK_DTS := 1 2 3 6 7 9
PK_OBJS := $(patsubst %,$(OBJ)/dt_launch_dt%.o,$(PK_DTS))
$(OBJ)/xalm_hip.o: $(HIP_SRC) $(HIP_HDR)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $(HIP_SRC)
$(OBJ)/dt_launch_dt%.o: xalm_amd/csrc/dt_launch.hip $(HIP_HDR)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -DPK_DT=$* -c -o $@ $<
$(LIB)/libxalm_hip.so: $(OBJ)/xalm_hip.o $(PK_OBJS)
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^

HOST_LIB_SRC := $(filter-out xalm_amd/host/main.cpp,$(HOST_SRC))
$(LIB)/libxalm_host.so: $(HOST_LIB_SRC) $(HOST_HDR) $(LIB)/libxalm_hip.so
	$(CXX) $(HOSTFLAGS) -fopenmp -shared -o $@ $(HOST_LIB_SRC) -L$(LIB) -lxalm_hip -Wl,-rpath,'$$ORIGIN'

$(BIN)/xalm: xalm_amd/host/main.cpp $(LIB)/libxalm_host.so
	@mkdir -p $(BIN)
	$(CXX) $(HOSTFLAGS) -o $@ xalm_amd/host/main.cpp -L$(LIB) -lxalm_host -lxalm_hip -Wl,-rpath,'$$ORIGIN/../lib'

clean:
	rm -rf $(LIB) $(BIN) $(OBJ)
	$(MAKE) -C oracle clean
