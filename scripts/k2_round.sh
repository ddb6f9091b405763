#!/bin/bash
# Pair-kernel iteration: parity tests, probe timing, kernel trace, PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
STAGES="${STAGES:-tests}" bash scripts/gpu_round.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k2prof -o run -- python3 -u scripts/k2_probe.py > gpurun_out/k2prof.log 2>&1 || exit $?
if [ -n "$PMC" ]; then
  timeout -k 10 600 bash scripts/pmc.sh gpurun_out/pmc_gate "$PMC" -- python3 -u scripts/k2_probe.py --reps 1 > gpurun_out/pmc_gate.log 2>&1 || exit $?
fi
exit 0
