#!/bin/bash
# Build the working tree into galah_amd/lib_alt (B) and HEAD into galah_amd/lib (A).
cd "$(dirname "$0")/.." || exit 2
make -s -j8 -C galah_amd/csrc ARCH=gfx950 OUT=$PWD/galah_amd/lib_alt/libgalahgpu.so OBJDIR=$PWD/galah_amd/build_alt 2>&1 | grep -v hip-link
git stash -q || exit 1
touch galah_amd/csrc/*.hip galah_amd/csrc/*.cpp
make -s -j8 -C galah_amd/csrc ARCH=gfx950 2>&1 | grep -v hip-link
git stash pop -q
touch galah_amd/csrc/*.hip galah_amd/csrc/*.cpp
