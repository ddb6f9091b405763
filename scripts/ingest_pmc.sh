#!/bin/bash
# PMC passes over one device-inflate call on C2-like files (1,000 x 3 Mbp
# gzip FASTA, scripts/inflate_probe.py) for every ingest kernel: the slot
# upload, block-start search, staged and global decodes, expand, resolve,
# CRC, the three parse passes and K1.  One lane (GALAHGPU_GZ_LANES=1: the
# kernels of two lanes would share the counters' time) and one rocprofv3 run
# per counter set (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE each in a
# pass of their own).  Summarised by scripts/ingest_pmc_model.py.
# usage: scripts/ingest_pmc.sh <outdir> [n_files]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp PROBE_MODES=device GALAHGPU_GZ_LANES=1
out=$1
n=${2:-1000}
mkdir -p "$out"
rx='inflate_|parse_|slot_upload|sketch_candidates|sketch_finalize'
sets=(
  "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT"
  "GRBM_GUI_ACTIVE FETCH_SIZE"
  "GRBM_GUI_ACTIVE WRITE_SIZE"
)
i=0
for s in "${sets[@]}"; do
  i=$((i+1))
  echo "== pmc pass $i: $s"
  timeout -s KILL 280 rocprofv3 --pmc $s --kernel-include-regex "$rx" --output-format csv -d "$out/p$i" -o p$i -- python3 -u scripts/inflate_probe.py $n 1 > "$out/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 1 "$out/p$i.log"
  [ $rc -eq 0 ] || exit $rc
done
