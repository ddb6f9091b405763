# round 2, call ab: row-range (Bloom-filtered) K2 index for multi-device
# calls -- multi-device + parity tests, then the sharded C3 bench on one GPU
# (2 / 4 / 8 shards) with the row-range index on and off
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2ab && mkdir -p $out || exit 2
timeout -k 10 600 python3 -u -m pytest tests/test_multi_device.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -n 3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for dv in 0,0 0,0,0,0 0,0,0,0,0,0,0,0; do
  for rg in 1 0; do
    GALAHGPU_INDEX_RANGE=$rg timeout -k 10 300 python3 -u bench.py --devices $dv --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_${dv}_r$rg.json 2> $out/bench_${dv}_r$rg.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['phase_ms'], d['pairs_found'])" $out/bench_${dv}_r$rg.json "$dv range=$rg"
  done
done
