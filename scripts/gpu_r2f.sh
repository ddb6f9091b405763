# round 2, call f: K1 PMC at C5 vs C3 (why C5 runs 25% fewer k-mers/s)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2f || exit 2
rx='sketch_candidates'
pass() { # name config counters...
  local n=$1 cfg=$2; shift 2
  echo "== $n"
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$rx" --output-format csv -d gpurun_out/r2f/$n -o $n -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --config $cfg > gpurun_out/r2f/$n.log 2>&1
  local rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
timeout -k 10 120 rocprofv3 -L > gpurun_out/r2f/counters.txt 2>&1 || exit $?
P4=""
for x in SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA; do
  grep -qw "$x" gpurun_out/r2f/counters.txt && P4="$P4 $x"
done
echo "p4 counters:$P4"
pass c5_p1 c5 GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES &&
pass c5_p3 c5 GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY TCC_HIT_sum TCC_MISS_sum &&
pass c5_p4 c5 GRBM_GUI_ACTIVE $P4 &&
pass c3_p4 c3 GRBM_GUI_ACTIVE $P4 &&
pass c3_p1 c3 GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES
