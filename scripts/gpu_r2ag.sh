# round 2, call ag: per-peer replication streams -- multi-device tests, sharded C3 bench on one GPU
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2ag && mkdir -p $out || exit 2
timeout -k 10 600 python3 -u -m pytest tests/test_multi_device.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -n 2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for dv in 0,0 0,0,0,0 0,0,0,0,0,0,0,0; do
  timeout -k 10 300 python3 -u bench.py --devices $dv --steps 10 --warmup 2 --no-cpu-baseline > $out/bench_$dv.json 2> $out/bench_$dv.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['phase_ms'], d['pairs_found'])" $out/bench_$dv.json "$dv"
done
