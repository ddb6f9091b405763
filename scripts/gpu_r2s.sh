# round 2, call s: K1 canonical min through VCC (v_cmp_lt_u64_e32 + v_cndmask_b32_e32) vs compiler choice
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2s || exit 2
b() { local n=$1 lib=$2; shift 2; echo "== $n"
  GALAHGPU_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/r2s/$n.json 2> gpurun_out/r2s/$n.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['roofline']['kernels'][0]['avg_ms'])" gpurun_out/r2s/$n.json; }
A=galah_amd/lib/libgalahgpu.so; B=galah_amd/lib_g1/libgalahgpu.so
echo "== tests B" && GALAHGPU_LIB=$B timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sketch or edge or other_k or synthetic or runs" > gpurun_out/r2s/tests.log 2>&1; rc=$?; tail -n 2 gpurun_out/r2s/tests.log; [ $rc -eq 0 ] || exit $rc
b a1 $A && b b1 $B && b a2 $A && b b2 $B && b a3 $A && b b3 $B
