# round 2, call t: evidence at HEAD -- full GPU suite, smoke, C3 bench with the CPU baseline, and the
# rocprofv3 kernel-trace stats of the same bench command (profiles/ must agree with the bench line)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2t || exit 2
echo "== tests" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r2t/tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r2t/tests.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2t/smoke.log 2>&1 || exit $?
tail -n 1 gpurun_out/r2t/smoke.log
echo "== bench" && timeout -k 10 600 python3 -u bench.py > gpurun_out/r2t/bench.json 2> gpurun_out/r2t/bench.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline']['kernels'][0]['peak_stale'], d['cpu_baseline']['value'])" gpurun_out/r2t/bench.json
echo "== trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2t/trace -o c3 -- python3 bench.py --no-cpu-baseline > gpurun_out/r2t/trace.log 2>&1
