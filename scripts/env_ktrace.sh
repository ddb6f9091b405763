#!/bin/bash
# Kernel durations (rocprofv3 --kernel-trace --stats) of device-inflate calls
# on C2-like files under different environment settings, one process each
# (for knobs read once per process).  usage:
#   scripts/env_ktrace.sh OUTDIR FILES 'name:K=V,K=V' ['name:...' ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp PROBE_MODES=device GALAHGPU_GZ_LANES=1
out=$1; n=$2; shift 2
mkdir -p "$out"
for spec in "$@"; do
  name=${spec%%:*}; kv=${spec#*:}
  (
    IFS=',' read -ra pairs <<< "$kv"
    for p in "${pairs[@]}"; do [ -n "$p" ] && export "$p"; done
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$name$RANDOM" -o kt -- python3 -u scripts/inflate_probe.py $n 2 > "$out/$name.log" 2>&1
  ) || exit $?
  tail -n 1 "$out/$name.log"
done
