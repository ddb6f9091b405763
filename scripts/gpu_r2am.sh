# round 2, call am: K1 wave-aggregated queue push (GG_K1_WAVEPUSH) -- parity on lib_gW, C3/C5 A/B vs lib (HEAD)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2am && mkdir -p $out || exit 2
GALAHGPU_LIB=galah_amd/lib_gW/libgalahgpu.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -n 2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in c3 c5; do
    for v in lib lib_gW; do
      GALAHGPU_LIB=galah_amd/$v/libgalahgpu.so timeout -k 10 300 python3 -u bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_${cfg}_${v}_$r.json 2> $out/bench_${cfg}_${v}_$r.err || exit $?
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['avg_launch_ms'])" $out/bench_${cfg}_${v}_$r.json "$cfg $v"
    done
  done
done
