# round 2, call g: K1 segments inside runs; parity (default and G forced), C5/C3 benches, C5 PMC pass
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2g || exit 2
b() { # name env...
  local n=$1; shift
  echo "== $n"; env "$@" timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $BARGS > gpurun_out/r2g/$n.json 2> gpurun_out/r2g/$n.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['phase_ms'], d['roofline']['kernels'][0]['avg_ms'])" gpurun_out/r2g/$n.json
}
echo "== tests" && timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2g/tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r2g/tests.log; [ $rc -eq 0 ] || exit $rc
echo "== tests G=1" && GALAHGPU_K1_GROUP=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2g/tests_g1.log 2>&1; rc=$?; tail -n 3 gpurun_out/r2g/tests_g1.log; [ $rc -eq 0 ] || exit $rc
BARGS="--config c5"
b c5_g1 GALAHGPU_K1_GROUP=1 && b c5_g4 GALAHGPU_K1_GROUP=4 &&
BARGS="" && b c3_g4 GALAHGPU_K1_GROUP=4 && b c3_g1 GALAHGPU_K1_GROUP=1 &&
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex sketch_candidates --output-format csv -d gpurun_out/r2g/c5_p1 -o c5_p1 -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --config c5 > gpurun_out/r2g/c5_p1.log 2>&1
