# Builds the gfx950 shared library behind include/botorch_amd.h.
#   make            -> botorch_amd/libbotorch_amd.so
#   make oracle     -> (no native oracle: the oracle is torch fp64 on CPU)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function \
            -Wno-unused-variable -munsafe-fp-atomics
SRC := $(wildcard botorch_amd/csrc/*.hip)
CPPSRC := $(wildcard botorch_amd/csrc/*.cpp)
OBJ := $(patsubst botorch_amd/csrc/%.hip,build/%.o,$(SRC)) $(patsubst botorch_amd/csrc/%.cpp,build/%.o,$(CPPSRC))
CXX ?= g++
CXXFLAGS ?= -O3 -std=c++17 -fPIC -pthread -Wall
HDR := $(wildcard botorch_amd/csrc/*.h) include/botorch_amd.h
LIB := botorch_amd/libbotorch_amd.so
# the torch operators (TORCH_LIBRARY): host C++ against torch's ROCm headers,
# linked to the kernel library
TORCH_DIR ?= $(shell python3 -c "import os, torch; print(os.path.dirname(torch.__file__))")
TORCH_LIB := botorch_amd/libbotorch_amd_torch.so
TORCH_SRC := $(wildcard botorch_amd/csrc/torch/*.cpp)
TORCH_FLAGS := -O2 -std=c++17 -fPIC -shared -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 \
               -I$(TORCH_DIR)/include -I$(TORCH_DIR)/include/torch/csrc/api/include \
               -I/opt/rocm/include -Wall -Wno-unused-function

all: $(LIB) $(TORCH_LIB)

$(TORCH_LIB): $(TORCH_SRC) include/botorch_amd.h $(LIB)
	$(CXX) $(TORCH_FLAGS) $(TORCH_SRC) -o $@ -Lbotorch_amd -lbotorch_amd \
	  -L$(TORCH_DIR)/lib -ltorch -ltorch_cpu -lc10 -lc10_hip -ltorch_hip \
	  -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(TORCH_DIR)/lib

build/%.o: botorch_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# host-only native code (no device code): plain g++
build/%.o: botorch_amd/csrc/%.cpp $(HDR)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(OBJ) -pthread -o $@

# development probes (tools/bo_tools.h): the same sources with -DBO_TOOLS, into
# a tools-only library the tools/ scripts load; never part of the product
TOOLS_LIB := tools/libbotorch_amd_tools.so
TOOLS_OBJ := $(patsubst botorch_amd/csrc/%.hip,build/tools/%.o,$(SRC)) $(patsubst botorch_amd/csrc/%.cpp,build/tools/%.o,$(CPPSRC))

build/tools/%.o: botorch_amd/csrc/%.hip $(HDR)
	@mkdir -p build/tools
	$(HIPCC) $(HIPFLAGS) -DBO_TOOLS -c $< -o $@

build/tools/%.o: botorch_amd/csrc/%.cpp $(HDR)
	@mkdir -p build/tools
	$(CXX) $(CXXFLAGS) -DBO_TOOLS -c $< -o $@

tools: $(TOOLS_LIB)

$(TOOLS_LIB): $(TOOLS_OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(TOOLS_OBJ) -pthread -o $@

# qmc_kernel phase clocks (tools/qmc_phases.sh swaps it in for one run): the
# product objects with qmc.hip built -DBO_QMC_PHASES; never the product
PH_LIB := ab_libs/libP.so

$(PH_LIB): $(OBJ) botorch_amd/csrc/qmc.hip $(HDR)
	@mkdir -p build/ph ab_libs
	$(HIPCC) $(HIPFLAGS) -DBO_QMC_PHASES -c botorch_amd/csrc/qmc.hip -o build/ph/qmc.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(filter-out build/qmc.o,$(OBJ)) build/ph/qmc.o -pthread -o $@

qmc-phases: $(PH_LIB)

clean:
	rm -rf build $(LIB) $(TORCH_LIB) $(TOOLS_LIB) $(PH_LIB)

.PHONY: all clean tools qmc-phases
