# round 2, call y: K2HI A/B at C3 (lib_g00 = round-2 start of this session,
# lib = HEAD, lib_gH = HEAD + GG_K1_K2HI), parity of lib_gH
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2y && mkdir -p $out || exit 2
GALAHGPU_LIB=galah_amd/lib_gH/libgalahgpu.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "sketch or golden or edge" > $out/tests.log 2>&1; rc=$?; tail -n 2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in lib_g00 lib lib_gH; do
    GALAHGPU_LIB=galah_amd/$v/libgalahgpu.so timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_${v}_$r.json 2> $out/bench_${v}_$r.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['avg_launch_ms'])" $out/bench_${v}_$r.json $v
  done
done
