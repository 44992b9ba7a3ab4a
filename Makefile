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

all: $(LIB)

build/%.o: botorch_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# host-only native code (no device code): plain g++
build/%.o: botorch_amd/csrc/%.cpp $(HDR)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(OBJ) -pthread -o $@

clean:
	rm -rf build $(LIB)

.PHONY: all clean
