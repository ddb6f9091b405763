# round 2, call ad: row-range index v2 (blocked Bloom, fused fill, row-balanced parts):
# multi-device + parity tests, per-part K2 latency (C3, C4 shape), sharded C3 bench on one GPU
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2ad && mkdir -p $out || exit 2
timeout -k 10 600 python3 -u -m pytest tests/test_multi_device.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -n 3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for rg in 0 1; do
  GALAHGPU_INDEX_RANGE=$rg timeout -k 10 300 python3 -u scripts/k2_range_probe.py > $out/c3_r$rg.txt 2>&1 || exit $?
  grep '"M"' $out/c3_r$rg.txt | sed "s/^/c3 range=$rg /"
done
for rg in 0 1; do
  GALAHGPU_INDEX_RANGE=$rg timeout -k 10 400 python3 -u scripts/k2_range_probe.py --genomes 100000 --parts 1,8 --reps 3 > $out/c4_r$rg.txt 2>&1 || exit $?
  grep '"M"' $out/c4_r$rg.txt | sed "s/^/c4 range=$rg /"
done
for dv in 0,0,0,0 0,0,0,0,0,0,0,0; do
  timeout -k 10 300 python3 -u bench.py --devices $dv --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_$dv.json 2> $out/bench_$dv.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['phase_ms'], d['pairs_found'])" $out/bench_$dv.json "$dv"
done
