#!/bin/bash
# An alternate libgalahgpu.so for A/B runs (GALAHGPU_LIB=galah_amd/lib/ab/libgalahgpu_<name>.so):
# the HEAD objects with one source recompiled under extra flags.
#   scripts/ab_lib.sh <name> <source, e.g. inflate.hip> <flags...>
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
make -s -j8 -C galah_amd/csrc ARCH=gfx950 >/dev/null
mkdir -p galah_amd/lib/ab build_ab
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -mllvm \
  -pragma-unroll-threshold=1000000 "$@" -x hip -c galah_amd/csrc/$src -o build_ab/$src.o
objs=$(ls galah_amd/build/*.o | grep -v "/$src.o" | grep -v api_xcheck | grep -v "/pairs.hip.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o galah_amd/lib/ab/libgalahgpu_$name.so $objs build_ab/$src.o \
  -lz -lpthread -ldl
echo galah_amd/lib/ab/libgalahgpu_$name.so
