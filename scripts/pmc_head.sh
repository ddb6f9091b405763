#!/bin/bash
# PMC passes at HEAD over one C3 step (K1 + K2) and the FETCH_SIZE width
# calibration; each pass is its own rocprofv3 run (counter slots per pass are
# limited).  usage: scripts/pmc_head.sh <outdir> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
rx='sketch_candidates|sketch_finalize|pairs_gate|gate_build|gate_lo32'
sets=(
  "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
  "GRBM_GUI_ACTIVE FETCH_SIZE"
  "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY TCC_HIT_sum TCC_MISS_sum"
)
i=0
for s in "${sets[@]}"; do
  i=$((i+1))
  echo "== pmc pass $i: $s"
  timeout -s KILL 180 rocprofv3 --pmc $s --kernel-include-regex "$rx" --output-format csv -d "$out/p$i" -o p$i -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-files "$@" > "$out/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 2 "$out/p$i.log"
  [ $rc -eq 0 ] || exit $rc
done
echo "== fetch calibration"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$out/fetch" -o fetch -- ./scripts/ubench_fetch > "$out/fetch.log" 2>&1
rc=$?; echo "rc=$rc"; exit $rc
