#!/bin/bash
# Device-inflate ingest knobs A/B on C2-like files in one box call (each
# setting twice, alternating): GALAHGPU_GZ_BATCH_MB, GALAHGPU_GZ_COPY_THREADS,
# GALAHGPU_GZ_MMAP.  usage: scripts/inflate_ab.sh <outdir> "<setting>"...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp PROBE_MODES=device
out=$1; shift
mkdir -p "$out"
for rep in 1 2; do
  for st in "$@"; do
    tag=$(echo "$st" | tr ' =' '_-')
    echo "== $rep $st"
    env $st timeout -k 10 200 python3 -u scripts/inflate_probe.py ${PROBE_FILES:-1000} 4 > "$out/${tag}_$rep.log" 2>&1 || exit $?
    tail -n 1 "$out/${tag}_$rep.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['device']['s'])"
  done
done
