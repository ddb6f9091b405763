#!/bin/bash
# PMC passes (one rocprofv3 run per counter set) over a target command.
# usage: scripts/pmc.sh <outdir> <kernel-regex> -- cmd...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out=$1; rx=$2; shift 3
mkdir -p "$out"
sets=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  "FETCH_SIZE GRBM_GUI_ACTIVE"
  "TCC_HIT_sum TCC_MISS_sum"
)
i=0
for s in "${sets[@]}"; do
  i=$((i+1))
  [ -n "$PMC_SETS" ] && [ $i -gt "$PMC_SETS" ] && break
  echo "== pmc pass $i: $s"
  timeout -s KILL 120 rocprofv3 --pmc $s --kernel-include-regex "$rx" --output-format csv -d "$out/p$i" -o p$i -- "$@" > "$out/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 3 "$out/p$i.log"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
