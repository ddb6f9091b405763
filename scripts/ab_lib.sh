#!/bin/bash
# An alternate libgalahgpu.so for A/B runs (GALAHGPU_LIB=galah_amd/lib/ab/libgalahgpu_<name>.so):
# the HEAD objects with some sources recompiled under extra flags (every
# source that sees the flag must be listed, e.g. inflate.hip,inflate_host.cpp
# for a constant inflate_core.hpp shares between kernel and host).
#   scripts/ab_lib.sh <name> <source[,source...]> <flags...>
set -e
cd "$(dirname "$0")/.."
name=$1; srcs=$2; shift 2
make -s -j8 -C galah_amd/csrc ARCH=gfx950 >/dev/null
mkdir -p galah_amd/lib/ab build_ab
objs=$(ls galah_amd/build/*.o | grep -v api_xcheck | grep -v "/pairs.hip.o")
ab=""
for src in ${srcs//,/ }; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -mllvm \
    -pragma-unroll-threshold=1000000 "$@" -x hip -c galah_amd/csrc/$src -o build_ab/$src.o
  objs=$(echo "$objs" | grep -v "/$src.o")
  ab="$ab build_ab/$src.o"
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o galah_amd/lib/ab/libgalahgpu_$name.so $objs $ab -lz -lpthread -ldl
echo galah_amd/lib/ab/libgalahgpu_$name.so
