#!/bin/bash
# Kernel durations (rocprofv3 --kernel-trace --stats) of one device-inflate
# call on C2-like files per library build: HEAD and each alternate build
# (galah_amd/lib/ab/libgalahgpu_<name>.so).  One lane, so kernels do not share
# the GPU.  usage: scripts/ktrace_ab.sh OUTDIR FILES name [name ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp PROBE_MODES=device GALAHGPU_GZ_LANES=1
out=$1; n=$2; shift 2
mkdir -p "$out"
for name in head "$@" head; do
  if [ "$name" = head ]; then unset GALAHGPU_LIB; else export GALAHGPU_LIB=galah_amd/lib/ab/libgalahgpu_$name.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$name$RANDOM" -o kt -- python3 -u scripts/inflate_probe.py $n 2 > "$out/$name.log" 2>&1 || exit $?
  tail -n 1 "$out/$name.log"
done
