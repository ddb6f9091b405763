#!/bin/bash
# K1 grid A/B: the bench per GALAHGPU_K1_WG_PER_CU value, K1/finalize/K2 ms each.
#   CONFIGS="c3 c5" PASSES=2 STEPS=10 OUT=r3ai bash scripts/k1_grid_ab.sh 96 108 112 120 132
# (round 3 ran 56/112/224/28 at C3 and C5 -> profiles/r03_*; 96-132 at C3 -> profiles/r03_t/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out="gpurun_out/${OUT:-k1grid}"
mkdir -p "$out"
for pass in $(seq 1 "${PASSES:-1}"); do
  for w in "$@"; do
    for cfg in ${CONFIGS:-c3}; do
      log="$out/wg${w}_${cfg}_p$pass.log"
      GALAHGPU_K1_WG_PER_CU=$w timeout -k 10 300 python3 -u bench.py --config $cfg --steps "${STEPS:-10}" --warmup 2 \
        --no-cpu-baseline --no-files > "$log" 2>&1 || exit 1
      tail -n 1 "$log" > "${log%.log}.json"
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], sys.argv[4], d['ms_per_step'], d['kernel_ms_per_step'])" \
        "${log%.log}.json" "$pass" "$w" "$cfg"
    done
  done
done
