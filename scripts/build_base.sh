#!/bin/bash
# Build libgalahgpu.so of another revision (default HEAD) into
# galah_amd/lib_base/ for A/B runs against the working tree's galah_amd/lib/:
#   scripts/build_base.sh [rev]
#   STAGES="benchalt" ALT_LIB=galah_amd/lib_base/libgalahgpu.so scripts/gpu_round.sh
set -e
cd "$(dirname "$0")/.."
rev=${1:-HEAD}
wt=$(mktemp -d /tmp/gg_base.XXXXXX)
git worktree add -q --detach "$wt" "$rev"
trap 'git worktree remove --force "$wt"' EXIT
make -s -j8 -C "$wt/galah_amd/csrc" ARCH=gfx950 OUT="$PWD/galah_amd/lib_base/libgalahgpu.so" \
  OBJDIR="$wt/build" 2>&1 | grep -v "occupancy\|warnings generated\|launch_bounds\|^ *|\|^ *[0-9]* |" || true
git -C "$wt" rev-parse --short HEAD > galah_amd/lib_base/REV
echo "built $(cat galah_amd/lib_base/REV) -> galah_amd/lib_base/libgalahgpu.so"
