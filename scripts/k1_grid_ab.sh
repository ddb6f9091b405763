#!/bin/bash
# K1 grid A/B: C3 bench per GALAHGPU_K1_WG_PER_CU value (args), K1 avg ms each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in "$@"; do
  GALAHGPU_K1_WG_PER_CU=$w timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-files > gpurun_out/k1grid_$w.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/k1grid_$w.log').read().strip().splitlines()[-1]); print('wg/cu', $w, d['ms_per_step'], d['phase_ms'], d['roofline']['kernels'][0]['avg_ms'])"
done
