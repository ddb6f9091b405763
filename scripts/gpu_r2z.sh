# round 2, call z: evidence at HEAD -- C3 bench with the CPU baseline, the
# rocprofv3 kernel-trace stats of the same command, C5 and C4-shape benches
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2z && mkdir -p $out || exit 2
timeout -k 10 120 ./scripts/sort_bits_probe > $out/sort_bits.txt 2>&1; cat $out/sort_bits.txt
echo "== bench" && timeout -k 10 600 python3 -u bench.py > $out/bench_c3.json 2> $out/bench_c3.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline']['kernels'][0]['peak_stale'], d['cpu_baseline']['value'])" $out/bench_c3.json
echo "== trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o c3 -- python3 bench.py > $out/bench_c3_traced.json 2> $out/trace.log || exit $?
echo "== c5" && timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu-baseline > $out/bench_c5.json 2> $out/bench_c5.err || exit $?
echo "== c4" && timeout -k 10 600 python3 -u bench.py --config c4 --steps 2 --warmup 1 > $out/bench_c4.json 2> $out/bench_c4.err || exit $?
python3 -c "import json,sys; [print(f, json.load(open(f))['ms_per_step'], json.load(open(f))['value']) for f in sys.argv[1:]]" $out/bench_c5.json $out/bench_c4.json
