#!/bin/bash
# One gpurun call: parity tests, smoke, benches.  Stops at the first crash,
# abort or time limit (exit codes other than 0/1 from pytest, any non-zero
# from the others); plain test failures (pytest exit 1) still let the
# bench run so its numbers come back with the failure log.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
STAGES="${STAGES:-tests smoke bench1k bench}"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  return $rc
}
for st in $STAGES; do
  case $st in
    tests)
      run gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
      rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    smoke)
      run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench1k)
      run bench_1k 300 python -u bench.py --genomes 1000 --steps 3 --warmup 1 --no-cpu-baseline || exit $? ;;
    bench)
      run bench 600 python -u bench.py --steps 3 --warmup 1 || exit $? ;;
    benchalt)  # same bench against an alternate build (GALAHGPU_LIB)
      GALAHGPU_LIB="${ALT_LIB:?}" run bench_alt 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit $? ;;
    bench2r)
      run bench_2rank_gloo 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --genomes 2000 --dist-backend gloo || exit $? ;;
    k2)
      run k2_probe 300 python -u scripts/k2_probe.py || exit $? ;;
    pmc_k2)
      run pmc_k2 900 bash scripts/pmc.sh gpurun_out/pmc_k2 pairs_table -- python3 -u scripts/k2_probe.py --reps 1 || exit $? ;;
    pmc_k1)
      run pmc_k1 900 bash scripts/pmc.sh gpurun_out/pmc_k1 sketch_candidates -- python3 -u scripts/k2_probe.py --reps 1 || exit $? ;;
    counters)
      run counters 120 rocprofv3 -L || exit $? ;;
    prof)
      run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit $? ;;
  esac
done
exit 0
