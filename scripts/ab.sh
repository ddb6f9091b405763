#!/bin/bash
# A/B of two builds on the C3 bench (+ the GPU parity tests on the B build).
#   ALT_LIB=galah_amd/lib_alt/libgalahgpu.so bash scripts/ab.sh [pytest -k expr]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
ALT=${ALT_LIB:-galah_amd/lib_alt/libgalahgpu.so}
echo "== tests (B)"
GALAHGPU_LIB=$ALT timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${1:+-k "$1"} > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for r in 1 2; do
  echo "== bench A"
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-files > gpurun_out/ab_a$r.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_a$r.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['phase_ms'], d['roofline']['kernels'][0]['avg_ms'], d['roofline']['kernels'][1]['avg_ms'])"
  echo "== bench B"
  GALAHGPU_LIB=$ALT timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-files > gpurun_out/ab_b$r.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_b$r.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['phase_ms'], d['roofline']['kernels'][0]['avg_ms'], d['roofline']['kernels'][1]['avg_ms'])"
done
