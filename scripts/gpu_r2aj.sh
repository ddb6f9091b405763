# round 2, call aj: K1 tau-branch group size with the deferred exact test (lib = 4, lib_gG1 = 1, lib_gG2 = 2)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2aj && mkdir -p $out || exit 2
for v in lib_gG1 lib_gG2; do
GALAHGPU_LIB=galah_amd/$v/libgalahgpu.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "sketch or golden or edge or kmer" > $out/tests_$v.log 2>&1; rc=$?; tail -n 1 $out/tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for cfg in c3 c5; do
    for v in lib lib_gG1 lib_gG2; do
      GALAHGPU_LIB=galah_amd/$v/libgalahgpu.so timeout -k 10 300 python3 -u bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_${cfg}_${v}_$r.json 2> $out/bench_${cfg}_${v}_$r.err || exit $?
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['avg_launch_ms'])" $out/bench_${cfg}_${v}_$r.json "$cfg $v"
    done
  done
done
