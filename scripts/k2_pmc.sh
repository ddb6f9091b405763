#!/bin/bash
# PMC passes over one bench step (K1 and every K2 kernel: index scan/fill,
# the radix sort, runs, pairs), one rocprofv3 run per counter set.
# usage: scripts/k2_pmc.sh <outdir> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
rx='sketch_candidates|index_|onesweep'
sets=(
  "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_VMEM_RD"
  "GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
  "GRBM_GUI_ACTIVE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
  "GRBM_GUI_ACTIVE FETCH_SIZE"
)
i=0
for s in "${sets[@]}"; do
  i=$((i+1))
  echo "== pmc pass $i: $s"
  timeout -s KILL 240 rocprofv3 --pmc $s --kernel-include-regex "$rx" --output-format csv -d "$out/p$i" -o p$i -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-files "$@" > "$out/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 1 "$out/p$i.log"
  [ $rc -eq 0 ] || exit $rc
done
