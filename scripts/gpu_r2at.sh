# round 2, call at: final evidence at HEAD (fused run-table index pass) -- full GPU suite, smoke,
# issue model, C3 bench with the CPU baseline and the rocprofv3 stats of the same command
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2at && mkdir -p $out || exit 2
echo "== tests" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -n 2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -n 1 $out/smoke.log
echo "== bench" && timeout -k 10 600 python3 -u bench.py > $out/bench_c3.json 2> $out/bench_c3.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['cpu_baseline']['value'])" $out/bench_c3.json
echo "== trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o c3 -- python3 bench.py --no-cpu-baseline > $out/bench_c3_traced.json 2> $out/trace.log || exit $?
echo "== c5" && timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu-baseline > $out/bench_c5.json 2> $out/bench_c5.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" $out/bench_c5.json
