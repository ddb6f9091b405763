#!/bin/bash
# K1 workgroups per CU around 112 (whole resident rounds: 6 workgroups per CU at a time), C3, two passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/r3ai
for pass in 1 2; do
  for w in 96 108 112 120 132; do
    GALAHGPU_K1_WG_PER_CU=$w timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-files > gpurun_out/r3ai/wg${w}_p$pass.log 2>&1 || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/r3ai/wg${w}_p$pass.log').read().strip().splitlines()[-1]);print('$pass','$w',d['ms_per_step'],d['kernel_ms_per_step'])"
  done
done
