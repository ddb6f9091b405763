# round 2, call o: K1 tau-branch group size (4 / 2 / 1) and tau oversampling at C5 and C3, after the segment fix
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2o || exit 2
b() { local n=$1 lib=$2; shift 2; echo "== $n"
  GALAHGPU_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/r2o/$n.json 2> gpurun_out/r2o/$n.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['phase_ms']['sketch'], d['roofline']['kernels'][0]['avg_ms'])" gpurun_out/r2o/$n.json; }
L4=galah_amd/lib/libgalahgpu.so; L2=galah_amd/lib_g2/libgalahgpu.so; L1=galah_amd/lib_g1/libgalahgpu.so
echo "== tests g1" && GALAHGPU_LIB=$L1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sketch or edge or other_k or synthetic or runs" > gpurun_out/r2o/tests_g1.log 2>&1; rc=$?; tail -n 2 gpurun_out/r2o/tests_g1.log; [ $rc -eq 0 ] || exit $rc
b c5_g4 $L4 --config c5 && b c5_g2 $L2 --config c5 && b c5_g1 $L1 --config c5 && b c5_g4b $L4 --config c5 &&
GALAHGPU_TAU_OVER=1.1 b c5_g4_o110 $L4 --config c5 && GALAHGPU_TAU_OVER=1.1 b c5_g1_o110 $L1 --config c5 &&
b c3_g4 $L4 && b c3_g2 $L2 && b c3_g1 $L1 && b c3_g4b $L4
