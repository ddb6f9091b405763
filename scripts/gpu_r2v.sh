# round 2, call v: VALU issue costs (SGPR-sourced VOP3 forms, 64-bit min forms);
# K1 variants MINHI / MULHI: parity on the default build, then C3 bench A/B over
# lib_g00 (both off = previous HEAD), lib_g10, lib_g01, lib (both on)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2v && mkdir -p $out || exit 2
timeout -k 10 240 ./scripts/ubench_dual 8 > $out/dual8.txt 2>&1 || exit $?
echo "== tests"
GALAHGPU_LIB=galah_amd/lib_g11w/libgalahgpu.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -n 2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in lib_g00 lib_g10 lib_g01 lib_g11i0 lib lib_g11w; do
    GALAHGPU_LIB=galah_amd/$v/libgalahgpu.so timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_${v}_$r.json 2> $out/bench_${v}_$r.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['avg_launch_ms'])" $out/bench_${v}_$r.json $v
  done
done
