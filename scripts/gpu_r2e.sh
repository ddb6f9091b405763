# round 2, call e: K1 tau-branch granularity (G = 1 vs 4) and tau oversampling
# A/B at C5 and C3, then the parity suite with G = 1 forced everywhere
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2e || exit 2
b() { # name env...
  local n=$1; shift
  echo "== $n"; env "$@" timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $BARGS > gpurun_out/r2e/$n.json 2> gpurun_out/r2e/$n.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['phase_ms'], d['roofline']['kernels'][0]['avg_ms'])" gpurun_out/r2e/$n.json
}
BARGS="--config c5"
b c5_g4 GALAHGPU_K1_GROUP=4 && b c5_g1 GALAHGPU_K1_GROUP=1 && b c5_g1_o110 GALAHGPU_K1_GROUP=1 GALAHGPU_TAU_OVER=1.10 && b c5_g4_o110 GALAHGPU_K1_GROUP=4 GALAHGPU_TAU_OVER=1.10 &&
BARGS="" &&
b c3_g4 GALAHGPU_K1_GROUP=4 && b c3_g1 GALAHGPU_K1_GROUP=1 && b c3_g4_o125 GALAHGPU_K1_GROUP=4 GALAHGPU_TAU_OVER=1.25 &&
echo "== tests G=1" && GALAHGPU_K1_GROUP=1 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2e/tests_g1.log 2>&1; rc=$?; tail -n 3 gpurun_out/r2e/tests_g1.log; exit $rc
