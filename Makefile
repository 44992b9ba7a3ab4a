# Builds the gfx950 shared library behind include/botorch_amd.h.
#   make            -> botorch_amd/libbotorch_amd.so
#   make oracle     -> (no native oracle: the oracle is torch fp64 on CPU)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function \
            -Wno-unused-variable -munsafe-fp-atomics
SRC := $(wildcard botorch_amd/csrc/*.hip)
OBJ := $(patsubst botorch_amd/csrc/%.hip,build/%.o,$(SRC))
HDR := $(wildcard botorch_amd/csrc/*.h) include/botorch_amd.h
LIB := botorch_amd/libbotorch_amd.so

all: $(LIB)

build/%.o: botorch_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(OBJ) -o $@

clean:
	rm -rf build $(LIB)

.PHONY: all clean
