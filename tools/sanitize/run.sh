#!/bin/bash
# Host-code sanitizer runs (no GPU): ASan+UBSan and TSan builds of the engine's
# host side + micro-batcher + a randomized driver (tools/sanitize/host_fuzz.cpp),
# linked against the regular gfx950 kernel objects (never launched here).
set -e
cd "$(dirname "$0")/../.."
make -s -j8 >/dev/null
SRC="emqx_amd/csrc/engine.cpp emqx_amd/csrc/batcher.cpp tools/sanitize/host_fuzz.cpp"
OBJ="build/kernels.o build/shard.o build/routes.o build/acl.o"
INC="-D__HIP_PLATFORM_AMD__ -I/opt/rocm/include"
LIB="-L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -pthread"
g++ -std=c++17 -g -O1 -fno-omit-frame-pointer -fsanitize=address,undefined $INC $SRC $OBJ $LIB -o /tmp/tm_fuzz_asan
ASAN_OPTIONS=detect_leaks=1 UBSAN_OPTIONS=halt_on_error=1 /tmp/tm_fuzz_asan 20000
g++ -std=c++17 -g -O1 -fsanitize=thread $INC $SRC $OBJ $LIB -o /tmp/tm_fuzz_tsan
TSAN_OPTIONS=halt_on_error=1 /tmp/tm_fuzz_tsan 5000
