#!/bin/bash
# One gpurun call: any sequence of stages, each under its own time limit.
#   STAGES="tests smoke bench" OUT=r3a scripts/gpu_round.sh
# Logs go to gpurun_out/$OUT/<stage>.log.  The call stops at the first crash,
# abort or time limit (any non-zero exit; pytest's plain test failures, exit 1,
# still let later stages run so their numbers come back with the failure log).
# Stages that take extra arguments read them from the environment:
#   BENCH_ARGS   extra bench.py arguments for bench* stages (the C3 stage runs the files leg unless --no-files)
#   ALT_LIB      alternate libgalahgpu.so for benchalt (GALAHGPU_LIB)
#   TESTS        pytest selection for the tests stage (default: tests -m gpu)
#   PMC_ARGS     bench.py arguments for the pmc stage (default: one C3 step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT="gpurun_out/${OUT:-run}"
mkdir -p "$OUT"
STAGES="${STAGES:-tests smoke bench}"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "$OUT/$name.log"
  return $rc
}
bench() {  # name limit args...
  local name=$1 lim=$2; shift 2
  run "$name" "$lim" python3 -u bench.py "$@" $BENCH_ARGS || exit $?
  tail -n 1 "$OUT/$name.log" > "$OUT/$name.json"
}
for st in $STAGES; do
  case $st in
    tests)
      run gpu_tests 900 python3 -u -m pytest ${TESTS:-tests -m gpu} -v --timeout 300 --timeout-method thread
      rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    hostinfo)  # the host's CPUs as this process sees them (nproc, affinity, cgroup quota)
      run hostinfo 60 python3 -u scripts/host_cpus.py || exit $? ;;
    inflate)  # device gzip inflate tests (GALAHGPU_INFLATE=device)
      run gpu_tests_inflate 400 python3 -u -m pytest tests/test_inflate.py -m gpu -v --timeout 300 --timeout-method thread
      rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    inflate_probe)  # device vs host gzip inflate on C2-like files (reasons for a hand-back on stderr)
      GALAHGPU_INFLATE_DEBUG=1 run inflate_probe 600 python3 -u scripts/inflate_probe.py ${PROBE_FILES:-200} 3 || exit $? ;;
    pmc_inflate)  # instruction counters of the device inflate kernels (one pass: 8 SQ counters)
      export PROBE_MODES=device
      run pmc_inflate 120 timeout -s KILL 100 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU \
        SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex 'inflate_|parse_' \
        --output-format csv -d "$OUT/pmc_inflate" -o p -- python3 -u scripts/inflate_probe.py 100 1 || exit $? ;;
    inflate_prof)  # kernel trace + stats of the device inflate probe
      PROBE_MODES=device run inflate_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o inflate -- \
        python3 -u scripts/inflate_probe.py ${PROBE_FILES:-200} 2 || exit $? ;;
    files_trace)  # kernels and copies of device-inflate calls on C2-like files (GPU idle gaps between kernels)
      PROBE_MODES=device run files_trace 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
        -d "$OUT/files_trace" -o t -- python3 -u scripts/inflate_probe.py ${PROBE_FILES:-1000} 2 || exit $? ;;
    files_probe)  # device-inflate calls on C2-like files, no debug output (the bench's files leg alone)
      PROBE_MODES=device run files_probe 600 python3 -u scripts/inflate_probe.py ${PROBE_FILES:-1000} 3 || exit $? ;;
    smoke)
      run smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench)       bench bench_c3 600 --steps 20 --warmup 5 ;;
    bench_nocpu) bench bench_c3 300 --steps 20 --warmup 5 --no-cpu-baseline --no-files ;;
    bench_c2)    bench bench_c2 300 --config c2 --steps 10 --warmup 2 --no-cpu-baseline ;;
    bench_c4)    bench bench_c4 600 --config c4 --steps 3 --warmup 1 --no-cpu-baseline ;;
    bench_c5)    bench bench_c5 300 --config c5 --steps 10 --warmup 2 --no-cpu-baseline ;;
    bench_files) bench bench_files 600 --files --steps 3 --warmup 1 --no-cpu-baseline ;;
    benchalt|benchalt2)  # the C3 and C5 benches against an alternate build (ALT_LIB / ALT_LIB2)
      lib=$ALT_LIB; [ $st = benchalt2 ] && lib=$ALT_LIB2
      GALAHGPU_LIB="${lib:?}" bench ${st}_c3 300 --steps 20 --warmup 5 --no-cpu-baseline --no-files
      GALAHGPU_LIB="${lib:?}" bench ${st}_c5 300 --config c5 --steps 10 --warmup 2 --no-cpu-baseline ;;
    bench2r)  # the driver's launch shape on one GPU (two members of GPU 0)
      run bench_2rank 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 bench.py --gpus 2 --devices 0,0 --steps 5 --warmup 2 --no-cpu-baseline || exit $? ;;
    bench8r)  # the driver's 8-GPU launch shape on one GPU (eight members of GPU 0; ranks 1-7 join the barriers)
      run bench_8rank 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29513 bench.py --gpus 8 --devices 0,0,0,0,0,0,0,0 --steps 10 --warmup 3 --no-cpu-baseline \
        --no-files || exit $?
      tail -n 1 "$OUT/bench_8rank.log" > "$OUT/bench_8rank.json" ;;
    bench_dist)  # one process per GPU layout (--mode dist) at world 1: the per-rank sketch + row-tile pairs path
      bench bench_dist 300 --mode dist --steps 20 --warmup 5 --no-cpu-baseline --no-files ;;
    bench_dist2)  # --mode dist at world 2 on one GPU: gloo all-gather through host memory (RCCL refuses two ranks on one GPU)
      run bench_dist2 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29512 bench.py --gpus 2 --mode dist --dist-backend gloo --steps 10 --warmup 2 --no-cpu-baseline \
        --no-files || exit $?
      tail -n 1 "$OUT/bench_dist2.log" > "$OUT/bench_dist2.json" ;;
    bench_shards)  # one member's share of C3 at 8/4/2 GPUs (1250/2500/5000 genomes) on one device: per-launch fixed costs
      for g in 1250 2500 5000; do bench bench_g$g 200 --genomes $g --steps 30 --warmup 5 --no-cpu-baseline --no-files; done ;;
    prof)  # kernel trace + stats of the C3 bench (per-kernel averages for profiles/)
      run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c3 -- \
        python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-files || exit $? ;;
    prof_c5)
      run prof_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c5 -- \
        python3 -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline || exit $? ;;
    trace_c3)  # kernels and memory copies of C3 steps (timeline, host gaps)
      run trace_c3 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace_c3" -o t -- \
        python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-files || exit $? ;;
    trace_c5)  # kernels and memory copies of one C5 step (timeline of the sketch phase)
      run trace_c5 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace_c5" -o t -- \
        python3 -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline || exit $? ;;
    pmc)  # PMC passes at HEAD (scripts/pmc_head.sh)
      run pmc 900 bash scripts/pmc_head.sh "$OUT/pmc" ${PMC_ARGS:-} || exit $? ;;
    pmc_k2)  # K2 counters at C3 and C5 (scripts/k2_pmc.sh; summarised by scripts/k2_pmc_model.py)
      run pmc_k2_c3 1000 bash scripts/k2_pmc.sh "$OUT/pmc_k2_c3" || exit $?
      run pmc_k2_c5 1000 bash scripts/k2_pmc.sh "$OUT/pmc_k2_c5" --config c5 || exit $? ;;
    pmc_k1)  # K1 instruction counters at C3 and C5 (scripts/pmc.sh passes 1-2)
      PMC_SETS=2 run pmc_k1_c3 400 bash scripts/pmc.sh "$OUT/pmc_k1_c3" sketch_candidates -- \
        python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-files || exit $?
      PMC_SETS=2 run pmc_k1_c5 400 bash scripts/pmc.sh "$OUT/pmc_k1_c5" sketch_candidates -- \
        python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-files || exit $? ;;
    k1trace)  # first K1 launch of one C3 and one C5 step, per library in K1_LIBS
      for lib in ${K1_LIBS:-galah_amd/lib/libgalahgpu.so}; do
        tag=$(basename $(dirname $lib))
        for cfg in c3 c5; do
          GALAHGPU_LIB=$lib run k1trace_${tag}_$cfg 300 rocprofv3 --kernel-trace --output-format csv \
            -d "$OUT/k1trace_${tag}_$cfg" -o t -- python3 -u bench.py --config $cfg --steps 1 --warmup 0 \
            --no-cpu-baseline --no-files || exit $?
        done
      done ;;
    overhead)  # fixed cost of a multi-member call: 1 vs 8 members of GPU 0 on a small set, HEAD lib and ALT_LIB
      for lib in galah_amd/lib/libgalahgpu.so ${ALT_LIB:-}; do
        tag=$(basename $(dirname $lib))
        for devs in 0 0,0,0,0,0,0,0,0; do
          GALAHGPU_LIB=$lib bench overhead_${tag}_$(echo $devs | tr -cd , | wc -c) 300 --devices $devs --genomes 2000 \
            --genome-len 200000 --steps 30 --warmup 5 --no-cpu-baseline --no-files
        done
      done ;;
    ubench3)
      run ubench_vop3 120 ./scripts/ubench_vop3 8 && run ubench_vop3_w1 120 ./scripts/ubench_vop3 1 || exit $? ;;
    ubench)
      run ubench 300 ./scripts/ubench_dual || exit $? ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
exit 0
