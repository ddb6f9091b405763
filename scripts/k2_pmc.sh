#!/bin/bash
# PMC passes over one bench step for every K2 kernel of the default
# (bucketed) inverted index: index_scan, bucket_hist, bucket_base, index_fill,
# the 16-bit onesweep sort, bucket_bounds, index_bucket, index_pairs and the
# passing pairs' device sort (pair_keys, rocPRIM, pair_gather).  One
# rocprofv3 run per counter set (MI355X_MICROARCH.md: FETCH_SIZE and
# WRITE_SIZE each in a pass of their own).
# usage: scripts/k2_pmc.sh <outdir> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
rx='index_|bucket_|split_|superbin_|onesweep|pair_keys|pair_gather|sort|merge|scan'
sets=(
  "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_VMEM_RD"
  "GRBM_GUI_ACTIVE FETCH_SIZE"
  "GRBM_GUI_ACTIVE WRITE_SIZE"
  "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
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
