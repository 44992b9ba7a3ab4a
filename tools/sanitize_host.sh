#!/bin/bash
# Host-code sanitizer builds (the GPU pool refuses GPU sanitizers): the
# threaded box decomposition (csrc/boxdecomp.cpp) under ASan + UBSan and under
# TSan, driven by tests/host/boxdecomp_driver.cpp.  Outputs under build/san/.
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p build/san
SRC="botorch_amd/csrc/boxdecomp.cpp tests/host/boxdecomp_driver.cpp"
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
    -pthread $SRC -o build/san/boxdecomp_asan
g++ -std=c++17 -O1 -g -fsanitize=thread -pthread $SRC -o build/san/boxdecomp_tsan
ASAN_OPTIONS=detect_leaks=1 ./build/san/boxdecomp_asan
TSAN_OPTIONS=halt_on_error=1 ./build/san/boxdecomp_tsan
